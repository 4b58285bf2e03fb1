#!/bin/bash
# round 3, call g3l: pass-R step variant (SA_RV_V2): parity with it, then A/B at 1 and 5 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3l
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
SA_RV_V2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread > $O/parity_v2.log 2>&1 || exit 1
B="python -u bench.py --steps 12 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B --contexts 1 --batches 1 --steps 4 > $O/c1_v0.json 2> $O/c1_v0.err || exit 2
SA_RV_V2=1 timeout -k 10 300 $B --contexts 1 --batches 1 --steps 4 > $O/c1_v2.json 2> $O/c1_v2.err || exit 3
timeout -k 10 300 $B > $O/c5_v0.json 2> $O/c5_v0.err || exit 4
SA_RV_V2=1 timeout -k 10 300 $B > $O/c5_v2.json 2> $O/c5_v2.err || exit 5
