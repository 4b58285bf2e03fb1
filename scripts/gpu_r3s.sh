#!/bin/bash
# round 2, call r3s: rblock chunk carries guessed in parallel (k_rb_guess) -- GPU suite, ONT lossy line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3s
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --ont --lossy 1.15 --e2e-batches 0 --steps 16 > $O/b_ont.json 2> $O/b_ont.err || exit 2
