#!/bin/bash
# round 6, call r6z8: the R-Block speculative pass on n workgroups per CU
# taking 64 chunks at a time from a counter (SA_RB_SPEC_WG=n) against one grid
# of a lane per chunk (0, default): the R-Block GPU tests, then the ONT-shape
# lossy batch alone, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z8}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "rblock or ont" > $O/tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
B="bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10"
for rep in 1 2; do
    for n in 0 2 4; do
        step wg${n}_$rep env SA_RB_SPEC_WG=$n timeout -k 10 300 python -u $B > $O/wg${n}_$rep.json 2>> $O/ont.err
    done
done
