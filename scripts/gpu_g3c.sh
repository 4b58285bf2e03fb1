#!/bin/bash
# round 3, call g3c: the reference (HASH index) block path + its CLI on the GPU against the oracle; then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3c
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_align.py -x -v --timeout 240 --timeout-method thread > $O/align.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_align.py > $O/tests.log 2>&1 || exit 2
