#!/bin/bash
# round 3, call g4i: process teardown after page-locked host memory / device memory (exit_probe)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4i
mkdir -p $O
cd $R
timeout -k 10 400 python -u scripts/exit_probe.py > $O/exit_probe.txt 2>&1 || exit 1
