#!/bin/bash
# round 4, call r4z7: the long AUX runs and MD5 on every third CU
# (SA_LONG_CU_EVERY=3) against every fourth (the default): the bench 4 / 3 /
# 4 / 3 on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z7}
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
step bench_e4a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_e4a.json 2> $O/bench_e4a.err
SA_LONG_CU_EVERY=3 step bench_e3a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_e3a.json 2> $O/bench_e3a.err
step bench_e4b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_e4b.json 2> $O/bench_e4b.err
SA_LONG_CU_EVERY=3 step bench_e3b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_e3b.json 2> $O/bench_e3b.err
