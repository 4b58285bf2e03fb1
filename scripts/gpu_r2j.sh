#!/bin/bash
# round 2, call j: 2-pass radix sorts (10/9-bit digits), allocation slack -- GPU tests, C=4/5 bench, traced e2e
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2j
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --contexts 4 --cpu-seconds 0 --e2e-batches 0 > $O/c4.json 2> $O/c4.err || exit 2
SA_TRACE=1 timeout -k 10 900 python -u bench.py --contexts 5 --cpu-seconds 0 --e2e-log $O/e2e_trace.log > $O/c5.json 2> $O/c5.err || exit 3
