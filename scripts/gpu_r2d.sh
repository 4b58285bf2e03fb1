#!/bin/bash
# round 2, call d: shared front scratch (fronts one at a time) -- 1/2/3 contexts
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for C in 2 3; do
  timeout -k 10 600 python -u bench.py --contexts $C --cpu-seconds 0 --no-verify > $O/c$C.json 2> $O/c$C.err || exit 2
done
SA_CODER_WAVES=2 SA_CODER_LDS=61440 timeout -k 10 600 python -u bench.py --contexts 3 --cpu-seconds 0 --no-verify > $O/c3_w2.json 2> $O/c3_w2.err || exit 3
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- \
    python3 -u $R/bench.py --contexts 3 --steps 6 --warmup 0 --batches 3 --cpu-seconds 0 --no-verify \
    > $O/prof_c3.json 2> $O/prof_c3.err || exit 5
