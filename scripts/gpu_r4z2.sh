#!/bin/bash
# round 4, call r4z2: pass R fed through the scalar memory path
# (SA_RV_VARIANT=4: the lanes publish (reciprocal, record) pairs into a
# per-wave ring, s_load_dwordx16 glc reads them 8 symbols at a time, 10 SALU a
# step, no v_readlane): the parity suite with it, then the bench 0 / 4 / 0 / 4
# on the same inputs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z2}
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
SA_RV_VARIANT=4 step parity_v4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity_v4.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_v0a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0a.json 2> $O/bench_v0a.err
SA_RV_VARIANT=4 step bench_v4a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v4a.json 2> $O/bench_v4a.err
step bench_v0b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v0b.json 2> $O/bench_v0b.err
SA_RV_VARIANT=4 step bench_v4b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_v4b.json 2> $O/bench_v4b.err
