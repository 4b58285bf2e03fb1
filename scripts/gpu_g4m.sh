#!/bin/bash
# round 3, call g4m: contexts per GPU on the tree with the faster front (g4l): 5 vs 6, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4m
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
for i in 1 2; do
    timeout -k 10 300 $B --contexts 6 > $O/c6_$i.json 2> $O/c6_$i.err || exit 1
    timeout -k 10 300 $B --contexts 5 > $O/c5_$i.json 2> $O/c5_$i.err || exit 2
done
