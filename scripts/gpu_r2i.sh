#!/bin/bash
# round 2, call i: 4-byte coder records -- GPU tests, C=4 / C=5 bench, traced end-to-end
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2i
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --contexts 4 --cpu-seconds 0 --e2e-batches 0 > $O/c4.json 2> $O/c4.err || exit 2
timeout -k 10 600 python -u bench.py --contexts 5 --cpu-seconds 0 --e2e-batches 0 > $O/c5.json 2> $O/c5.err || exit 3
SA_TRACE=1 timeout -k 10 900 python -u bench.py --contexts 4 --cpu-seconds 0 --no-verify --steps 2 --warmup 1 --e2e-log $O/e2e_trace.log > $O/c4_e2e.json 2> $O/c4_e2e.err || exit 4
