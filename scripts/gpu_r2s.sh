#!/bin/bash
# round 2, call s: HASH index + alignment GPU parity, full GPU suite, HASH bench, default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py -x -v --timeout 300 --timeout-method thread > $O/tests_hash.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
timeout -k 10 600 python -u scripts/bench_hash.py > $O/hash.json 2> $O/hash.err || exit 3
timeout -k 10 600 python -u bench.py --e2e-batches 0 > $O/bench.json 2> $O/bench.err || exit 4
