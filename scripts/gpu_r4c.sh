#!/bin/bash
# round 4, call r4c: the GPU suite, smoke, the profile set (kernel stats + PMC,
# inputs written first by a process that never touches the GPU), the default
# bench with all legs.  A step that ends in a signal, a time limit or an abort
# ends the call; an ordinary failure (exit 1) is recorded and the next step runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4c}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
step() {   # step NAME CMD...: run, record the exit status, stop the call on a hard failure
    local name=$1; shift
    "$@"; local rc=$?
    echo "$name rc=$rc" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc ${PYTEST_ARGS} > $O/tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
if [ -z "$NO_PROF" ]; then
    TAG=$TAG/prof_set step profile bash scripts/gpu_r4b.sh
fi
step bench timeout -k 10 1000 python -u bench.py --e2e-log $O/e2e.log ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err
