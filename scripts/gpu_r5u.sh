#!/bin/bash
# round 5, call r5u: R-Block chunk length (SA_RB_CHUNK = 8192 / 4096 / 2048):
# the lossy GPU parity tests with 2048-byte chunks, then same-call A/B of the
# ONT-shape lossy batch (bench.py --ont --lossy 1.15), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5u}
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
SA_RB_CHUNK=2048 step lossy_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "lossy or rblock or long" -o cache_dir=/tmp/pyc > $O/lossy_tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
for rep in 1 2; do
    for ch in 8192 4096 2048; do
        SA_RB_CHUNK=$ch step ont_$ch timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_${ch}_$rep.json 2>> $O/ont.err
        echo "{\"chunk\": $ch, \"rep\": $rep, \"line\": $(tail -1 $O/ont_${ch}_$rep.json)}" >> $O/ab_all.jsonl
    done
done
