#!/bin/bash
# round 2, call c: 4-chain pass-R workgroups (one per CU) + s_setprio; pipelined bench variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --contexts 1 --cpu-seconds 0 --no-verify > $O/c1.json 2> $O/c1.err || exit 2
timeout -k 10 600 python -u bench.py --contexts 2 --cpu-seconds 0 --no-verify > $O/c2.json 2> $O/c2.err || exit 3
SA_CHAIN_PRIO=0 timeout -k 10 600 python -u bench.py --contexts 2 --cpu-seconds 0 --no-verify > $O/c2_noprio.json 2> $O/c2_noprio.err || exit 4
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- \
    python3 -u $R/bench.py --contexts 2 --steps 4 --warmup 0 --batches 2 --cpu-seconds 0 --no-verify \
    > $O/prof_c2.json 2> $O/prof_c2.err || exit 5
