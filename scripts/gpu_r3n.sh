#!/bin/bash
# round 2, call r3n: 7-bit radix digits (SEQ 20 bits = 7+7+7 instead of 8+8+8): GPU suite, A/B against 8-bit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3n
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 24"
timeout -k 10 600 $B > $O/b_db7.json 2> $O/b_db7.err || exit 2
SA_SORT_MIN_DB=8 timeout -k 10 600 $B > $O/b_db8.json 2> $O/b_db8.err || exit 3
timeout -k 10 600 $B > $O/b_db7b.json 2> $O/b_db7b.err || exit 4
