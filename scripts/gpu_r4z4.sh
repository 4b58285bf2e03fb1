#!/bin/bash
# round 4, call r4z4: the pass-R step with the 48 v_readlane of sixteen steps
# batched (SA_RV_VARIANT=6) against eight steps (5, the default): the parity
# suite with 6, then the bench 5 / 6 / 5 / 6 on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z4}
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
SA_RV_VARIANT=6 step parity_v6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity_v6.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_v5a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5a.json 2> $O/bench_v5a.err
SA_RV_VARIANT=6 step bench_v6a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v6a.json 2> $O/bench_v6a.err
step bench_v5b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v5b.json 2> $O/bench_v5b.err
SA_RV_VARIANT=6 step bench_v6b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v6b.json 2> $O/bench_v6b.err
