#!/bin/bash
# round 3, call g3j: bench A/B -- k_emit_sq16 vs the wave kernel, 4 / 5 / 6 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3j
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/base.json 2> $O/base.err || exit 1
SA_EMIT_WAVE=1 timeout -k 10 300 $B > $O/wave.json 2> $O/wave.err || exit 2
timeout -k 10 300 $B --contexts 4 > $O/c4.json 2> $O/c4.err || exit 3
timeout -k 10 300 $B --contexts 6 > $O/c6.json 2> $O/c6.err || exit 4
