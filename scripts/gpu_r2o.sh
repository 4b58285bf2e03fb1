#!/bin/bash
# round 2, call o: bucketed BASE_MODEL replay -- GPU tests, bench default (32 steps) vs the full sort
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2o
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --cpu-seconds 0 --e2e-batches 0 > $O/bkt.json 2> $O/bkt.err || exit 2
SA_SEQ_FULLSORT=1 timeout -k 10 600 python -u bench.py --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/full.json 2> $O/full.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 12 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 4
