#!/bin/bash
# round 2, call x: A/B of the MD5 kernel against the front on one box (pipelined LDS reads, s_setprio),
# then the default bench with the end-to-end leg (pinned arena text windows, per-batch CLI trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2x
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "golden or stage_text or cli" > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 16"
timeout -k 10 600 $B > $O/b_def.json 2> $O/b_def.err || exit 2
SA_MD5_PIPE=0 timeout -k 10 600 $B > $O/b_nopipe.json 2> $O/b_nopipe.err || exit 3
SA_MD5_PRIO=0 timeout -k 10 600 $B > $O/b_prio0.json 2> $O/b_prio0.err || exit 4
SA_MD5_PIPE=0 SA_MD5_PRIO=0 timeout -k 10 600 $B > $O/b_nopipe_prio0.json 2> $O/b_nopipe_prio0.err || exit 5
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 6
