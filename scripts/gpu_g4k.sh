#!/bin/bash
# round 3, call g4k: the final-tree measurement set (round-3 end): the GPU suite in one process, the default bench (all legs),
# rocprofv3 kernel stats, PMC traffic (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4k
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 3
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u $R/bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/prof_bench.json 2> $O/prof_bench.err || exit 5
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 6
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/pmc_write.json 2> $O/pmc_write.err || exit 7
