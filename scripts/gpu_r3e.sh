#!/bin/bash
# round 2, call r3e: with the FIFO front: contexts 4 / 5 / 6 and pass-R priority off, one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3e
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 24"
timeout -k 10 600 $B > $O/b_c5.json 2> $O/b_c5.err || exit 1
timeout -k 10 600 $B --contexts 6 > $O/b_c6.json 2> $O/b_c6.err || exit 2
timeout -k 10 600 $B --contexts 4 > $O/b_c4.json 2> $O/b_c4.err || exit 3
SA_CHAIN_PRIO=0 timeout -k 10 600 $B > $O/b_prio0.json 2> $O/b_prio0.err || exit 4
