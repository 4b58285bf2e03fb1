#!/bin/bash
# round 2, call k: grid-stride per-read kernels, 9-bit digit cap -- GPU tests, C=5 bench + traced e2e, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2k
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
SA_TRACE=1 timeout -k 10 900 python -u bench.py --contexts 5 --cpu-seconds 0 --e2e-log $O/e2e_trace.log > $O/c5.json 2> $O/c5.err || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --contexts 5 --steps 4 --warmup 1 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 3
