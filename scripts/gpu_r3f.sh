#!/bin/bash
# round 2, call r3f: configs[4] shape (ONT-like SE long reads 10-50 kbp, -l 1.15) and the order-15 (Slevel 8)
# bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3f
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --ont --lossy 1.15 --e2e-batches 0 --steps 16 > $O/b_ont.json 2> $O/b_ont.err || exit 1
timeout -k 10 600 python -u bench.py --slevel 8 --e2e-batches 0 --steps 16 > $O/b_s8.json 2> $O/b_s8.err || exit 2
