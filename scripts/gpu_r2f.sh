#!/bin/bash
# round 2, call f: exact payload arenas, pass R defaults (VGPR, 4 chains / CU); 3 and 4 contexts; end-to-end CLI
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2f
mkdir -p $O
cd $R
df -h /tmp /dev/shm ${TMPDIR:-/tmp} > $O/df.txt 2>&1; free -g >> $O/df.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --contexts 3 > $O/c3.json 2> $O/c3.err || exit 2
timeout -k 10 900 python -u bench.py --contexts 4 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/c4.json 2> $O/c4.err || exit 3
