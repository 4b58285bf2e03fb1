#!/bin/bash
# round 2, call z: end-to-end A/B -- the CLI's encoder threads sleeping on their streams (SA_SYNC=block, the
# command line's default now) vs the runtime's default wait; four-slice reader
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2z
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0"
timeout -k 10 900 $B --e2e-log $O/e2e_block.log > $O/b_block.json 2> $O/b_block.err || exit 1
SA_SYNC=auto timeout -k 10 900 $B --e2e-log $O/e2e_auto.log > $O/b_auto.json 2> $O/b_auto.err || exit 2
