#!/bin/bash
# round 2, call e: VGPR-fed pass R (k_coder_rv) vs the scalar-load pass, 1 and 3 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2e
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --contexts 1 --cpu-seconds 0 --no-verify > $O/c1.json 2> $O/c1.err || exit 2
timeout -k 10 600 python -u bench.py --contexts 3 --cpu-seconds 0 --no-verify > $O/c3.json 2> $O/c3.err || exit 3
SA_CODER_VGPR=0 timeout -k 10 600 python -u bench.py --contexts 3 --cpu-seconds 0 --no-verify > $O/c3_salu.json 2> $O/c3_salu.err || exit 4
SA_CODER_WAVES=4 SA_CODER_LDS=83968 timeout -k 10 600 python -u bench.py --contexts 3 --cpu-seconds 0 --no-verify > $O/c3_w4.json 2> $O/c3_w4.err || exit 5
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- \
    python3 -u $R/bench.py --contexts 3 --steps 6 --warmup 0 --batches 3 --cpu-seconds 0 --no-verify \
    > $O/prof_c3.json 2> $O/prof_c3.err || exit 6
