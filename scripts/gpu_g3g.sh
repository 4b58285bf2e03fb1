#!/bin/bash
# round 3, call g3g: kernel stats of the bench with k_emit_sq16 (and the wave variant for A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3g
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 8 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/b16.json 2> $O/b16.err || exit 1
SA_EMIT_WAVE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/profw -o run -- python3 $R/bench.py --steps 8 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/bw.json 2> $O/bw.err || exit 2
