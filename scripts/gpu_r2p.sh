#!/bin/bash
# round 2, call p: bucketed BASE_MODEL replay with a prefetch ring + XCD mapping; MD5 priority at 32 steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2p
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/bkt.json 2> $O/bkt.err || exit 2
SA_MD5_PRIO=0 timeout -k 10 600 python -u bench.py --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/bkt_md5p0.json 2> $O/bkt_md5p0.err || exit 3
SA_SEQ_FULLSORT=1 SA_MD5_PRIO=0 timeout -k 10 600 python -u bench.py --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/full_md5p0.json 2> $O/full_md5p0.err || exit 4
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 12 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 5
SA_TRACE=1 timeout -k 10 900 python -u bench.py --cpu-seconds 0 --no-verify --steps 8 --e2e-log $O/e2e_trace.log > $O/e2e.json 2> $O/e2e.err || exit 6
