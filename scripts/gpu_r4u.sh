#!/bin/bash
# round 4, call r4u: the L passes at s_setprio 2 (SA_L_PRIO=1)
# against default priority: the bench
# A/B/A on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4u}
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
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_a.json 2> $O/bench_a.err
SA_L_PRIO=1 step bench_lprio timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_lprio.json 2> $O/bench_lprio.err
step bench_b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_b.json 2> $O/bench_b.err
