#!/bin/bash
# round 3, call g4e: knob sweep on the final tree (a hardware queue per stream): long-run / MD5 CU share (every 2nd /
# 8th CU), long-run grid (4 per CU), chain priority off, 4 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
i=0
for v in "SA_X=0" "SA_LONG_CU_EVERY=8" "SA_LONG_CU_EVERY=2" "SA_LONG_GRID=256" "SA_CHAIN_PRIO=0" "SA_X=1"; do
    i=$((i + 1))
    echo "$i $v" >> $O/variants.txt
    env $v timeout -k 10 300 $B > $O/b$i.json 2> $O/b$i.err || exit 2
done
timeout -k 10 300 $B --contexts 4 > $O/c4.json 2> $O/c4.err || exit 3
