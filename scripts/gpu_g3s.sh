#!/bin/bash
# round 3, call g3s: parity (new name-column test); bench A/B: hardware queues 4 vs 24, pass-R LDS reservation
# 82 / 64 / 0 KB, fused vs split name columns
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3s
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/base.json 2> $O/base.err || exit 2
GPU_MAX_HW_QUEUES=24 timeout -k 10 300 $B > $O/q24.json 2> $O/q24.err || exit 3
SA_CODER_LDS=65536 timeout -k 10 300 $B > $O/lds64.json 2> $O/lds64.err || exit 4
SA_CODER_LDS=0 timeout -k 10 300 $B > $O/lds0.json 2> $O/lds0.err || exit 5
SA_PREP_SPLIT=1 timeout -k 10 300 $B > $O/split.json 2> $O/split.err || exit 6
SA_LONG_CU_EVERY=1 timeout -k 10 300 $B > $O/every1.json 2> $O/every1.err || exit 8
timeout -k 10 300 $B > $O/base2.json 2> $O/base2.err || exit 7
