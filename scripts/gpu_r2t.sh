#!/bin/bash
# round 2, call t (rebuilt container): full GPU suite, smoke, default bench, kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2t
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --e2e-batches 0 > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 4
