#!/bin/bash
# round 4, call r4z6: the batched pass-R moves at issue priority 1 (the steps
# at 3; SA_RV_VARIANT=7) against all at 3 (5, the default for short reads):
# the bench 5 / 7 / 5 / 7 on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z6}
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
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_v5a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5a.json 2> $O/bench_v5a.err
SA_RV_VARIANT=7 step bench_v7a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v7a.json 2> $O/bench_v7a.err
step bench_v5b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5b.json 2> $O/bench_v5b.err
SA_RV_VARIANT=7 step bench_v7b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v7b.json 2> $O/bench_v7b.err
