#!/bin/bash
# round 3, call g4i: process teardown after page-locked host memory / device memory (exit_probe)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4i
mkdir -p $O
cd $R
timeout -k 10 400 python -u scripts/exit_probe.py > $O/exit_probe.txt 2>&1 || exit 1
# and the end-to-end legs with a plain input that fits one round dealt as equal batches (no ramp)
export TMPDIR=/tmp SA_NO_BUILD=1
sleep 10
timeout -k 10 900 python -u bench.py --steps 8 --cpu-seconds 0 --no-verify --e2e-log $O/e2e.log \
    > $O/bench_e2e.json 2> $O/bench_e2e.err || exit 2
