#!/bin/bash
# round 4, call r4v: the async tail (sa_run_input returns after pass R; the L
# passes and the assembly on a thread of the context).  The GPU suite with it
# on, then the bench A/B/A against SA_ASYNC_TAIL=0 on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4v}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step gpu_tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_a.json 2> $O/bench_a.err
SA_ASYNC_TAIL=0 step bench_sync timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_sync.json 2> $O/bench_sync.err
step bench_b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_b.json 2> $O/bench_b.err
