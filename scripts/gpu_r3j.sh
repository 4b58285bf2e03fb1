#!/bin/bash
# round 2, call r3j: configs[1] line -- 10 M x 150 bp SE, Slevel 8 (order 15, the "16-order" model)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3j
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --se --pairs 10000000 --slevel 8 --e2e-batches 0 --steps 16 > $O/b_c1_se_s8.json 2> $O/b_c1_se_s8.err || exit 1
