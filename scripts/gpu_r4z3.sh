#!/bin/bash
# round 4, call r4z3: the pass-R step with the 24 v_readlane of eight steps
# issued together ahead of their 64 SALU instructions (SA_RV_VARIANT=5): the
# parity suite with it, then the bench 0 / 5 / 0 / 5 on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z3}
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
SA_RV_VARIANT=5 step parity_v5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity_v5.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_v0a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0a.json 2> $O/bench_v0a.err
SA_RV_VARIANT=5 step bench_v5a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5a.json 2> $O/bench_v5a.err
step bench_v0b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0b.json 2> $O/bench_v0b.err
SA_RV_VARIANT=5 step bench_v5b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5b.json 2> $O/bench_v5b.err
