#!/bin/bash
# round 3, call g3p: e2e legs on a settled device (8 s idle before each), device buffers left to the exit
# vs --release
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3p
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --cpu-seconds 0 --no-verify --e2e-gz-blocks 0"
timeout -k 10 600 $B --e2e-log $O/e2e_exit.log > $O/exit.json 2> $O/exit.err || exit 1
timeout -k 10 600 $B --e2e-log $O/e2e_release.log --e2e-args=--release > $O/release.json 2> $O/release.err || exit 2
