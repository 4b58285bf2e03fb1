#!/bin/bash
# round 3, call g4o: the final tree, short set (round-3 end, the pool short of boxes): the GPU suite in one process, the default bench (all legs),
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4o
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 3
