#!/bin/bash
# round 3, call g4a: hardware queues per process (GPU_MAX_HW_QUEUES, preset to 4 on the boxes) with the resident-
# sized long-run grid: 4 / 8 / 12 / 24, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4a
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
for q in 4 8 12 24 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B > $O/q${q}_$RANDOM.json 2> $O/q$q.err || exit 2
done
