#!/bin/bash
# round 4, call r4x: the pass-R step variants (SA_RV_VARIANT: 1 -- the
# quotient correction after the frequency multiply, two multiplies on the
# dependent chain; 2 -- the same with the v_readlane between the chain's SALU
# steps): the parity suite with each, then the bench 0 / 1 / 2 / 0 on the same
# inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4x}
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
SA_RV_VARIANT=1 step parity_v1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity_v1.log 2>&1
SA_RV_VARIANT=2 step parity_v2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity_v2.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_v0a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0a.json 2> $O/bench_v0a.err
SA_RV_VARIANT=1 step bench_v1 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v1.json 2> $O/bench_v1.err
SA_RV_VARIANT=2 step bench_v2 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v2.json 2> $O/bench_v2.err
step bench_v0b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0b.json 2> $O/bench_v0b.err
