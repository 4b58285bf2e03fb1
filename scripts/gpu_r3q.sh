#!/bin/bash
# round 2, call r3q: final measurement set (packed SEQ keys) of the default bench -- full GPU suite + smoke, the default bench line
# (end to end included), rocprofv3 kernel trace + stats, PMC traffic (FETCH_SIZE and WRITE_SIZE passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3q
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --cpu-seconds 0 --e2e-batches 0 --steps 16 > $O/prof_bench.json 2> $O/prof_bench.err || exit 4
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/pmc_$C.json 2> $O/pmc_$C.err || exit 5
done
python3 scripts/pmc_traffic.py $(ls $O/pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/pmc_WRITE_SIZE/*counter_collection.csv | head -1) $O/traffic.json > $O/traffic.txt || exit 6
