#!/bin/bash
# round 3, call g3k: the GPU suite in one process, the GRCh38-sized HASH bench, the bench with e2e + gzip legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3k
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u scripts/bench_hash.py > $O/hash.json 2> $O/hash.err || exit 2
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 3
