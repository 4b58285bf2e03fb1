#!/bin/bash
# round 2, call b: kernel-trace timeline of the 2-context bench; HW-queue and
# batch-size variants of the pipelined bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2b
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- \
    python3 -u $R/bench.py --contexts 2 --steps 4 --warmup 2 --cpu-seconds 0 --no-verify \
    > $O/prof_c2.json 2> $O/prof_c2.err || exit 1
cd $R
GPU_MAX_HW_QUEUES=32 timeout -k 10 600 python -u bench.py --contexts 2 --cpu-seconds 0 --no-verify > $O/c2_q32.json 2> $O/c2_q32.err || exit 2
timeout -k 10 600 python -u bench.py --contexts 3 --pairs 2500000 --batches 6 --cpu-seconds 0 --no-verify > $O/c3_p25.json 2> $O/c3_p25.err || exit 3
