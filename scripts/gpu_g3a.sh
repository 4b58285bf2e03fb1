#!/bin/bash
# round 3, call g3a: baseline of the round-2 tree -- GPU suite, smoke, default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3a
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > $O/b.json 2> $O/b.err || exit 3
