#!/bin/bash
# round 2, call g: CLI without zero-filled buffers (end-to-end leg), 4 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "cli or exact or resident" > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --contexts 4 --cpu-seconds 0 > $O/c4.json 2> $O/c4.err || exit 2
