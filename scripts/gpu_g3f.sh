#!/bin/bash
# round 3, call g3f: hash + parity modules in one process (module-transition hang hunt), then the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3f
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_parity.py -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 2
