#!/bin/bash
# round 3, call g3o: device allocation / release cost probe; front phases vs contexts in flight (1, 2, 5) and
# pass-R priority off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3o
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 120 ./micro_run/alloc_probe2 5 33 2 > $O/alloc_5x33.txt 2>&1 || exit 1
timeout -k 10 120 ./micro_run/alloc_probe2 1 33 8 > $O/alloc_1x33.txt 2>&1 || exit 2
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B --contexts 1 --batches 1 --steps 3 > $O/c1.json 2> $O/c1.err || exit 3
timeout -k 10 300 $B --contexts 2 --batches 2 --steps 6 > $O/c2.json 2> $O/c2.err || exit 4
SA_CHAIN_PRIO=0 timeout -k 10 300 $B --steps 12 > $O/c5_prio0.json 2> $O/c5_prio0.err || exit 5
timeout -k 10 300 $B --steps 12 > $O/c5.json 2> $O/c5.err || exit 6
