#!/bin/bash
# round 2, call u: MD5 with a loader wave (bitop3 rounds), parallel reader + fast PE cut; GPU suite,
# default bench with the longer end-to-end stream, rocprofv3 kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2u
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 3
