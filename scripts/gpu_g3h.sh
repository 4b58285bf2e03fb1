#!/bin/bash
# round 3, call g3h: emit kernels with one context (little co-residence) A/B, and 5 contexts with k_emit_sq16<2> at 16 KB LDS
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3h
mkdir -p $O
cd /tmp
export TMPDIR=/tmp SA_NO_BUILD=1
B="python3 $R/bench.py --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1 -o run -- $B --contexts 1 --batches 1 --steps 3 > $O/b1.json 2> $O/b1.err || exit 1
SA_EMIT_WAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p1w -o run -- $B --contexts 1 --batches 1 --steps 3 > $O/b1w.json 2> $O/b1w.err || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p5 -o run -- $B --steps 8 > $O/b5.json 2> $O/b5.err || exit 3
