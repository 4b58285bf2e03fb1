#!/bin/bash
# round 2, call w: k_prep_sq16 (row per read) -- GPU suite, then A/B on one box: prep16 vs wave-per-read,
# x-span 8 vs 0 (name workload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2w
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 16 > $O/b_prep16.json 2> $O/b_prep16.err || exit 2
SA_PREP_WAVE=1 timeout -k 10 600 python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 16 > $O/b_prepwave.json 2> $O/b_prepwave.err || exit 3
timeout -k 10 600 python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 16 --x-span 0 > $O/b_x0.json 2> $O/b_x0.err || exit 4
