#!/bin/bash
# round 2, call r3m: the CU split under the pipeline (long AUX runs + MD5 on every Nth CU, pass R on the rest)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3m
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 24"
timeout -k 10 600 $B > $O/b_every4.json 2> $O/b_every4.err || exit 1
SA_LONG_CU_EVERY=8 timeout -k 10 600 $B > $O/b_every8.json 2> $O/b_every8.err || exit 2
SA_LONG_CU_EVERY=2 timeout -k 10 600 $B > $O/b_every2.json 2> $O/b_every2.err || exit 3
