#!/bin/bash
# round 5, call r5v: the final committed tree -- the GPU suite, smoke, the
# default bench with every leg (what the driver runs at the round's end).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5v}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf /dev/shm/seqarc_bench_*' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
