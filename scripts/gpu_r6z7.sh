#!/bin/bash
# round 6, call r6z7: k_emit_sq's listed (N / IUPAC) reads taken from a
# counter one at a time in long-read batches, against HEAD's static grid
# stride (ablib/, SA_LIB): the long-read / lossy GPU tests, the ONT-shape lossy
# batch alone twice each way, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z7}
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
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "rblock or ont or long or prep_row or read_counter or fetch_sizes or edge or golden or md5" > $O/tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
B="bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10"
for rep in 1 2; do
    step new_$rep timeout -k 10 300 python -u $B > $O/new_$rep.json 2>> $O/ont.err
    step head_$rep env SA_LIB=$R/ablib/libseqarc_amd_head.so timeout -k 10 300 python -u $B > $O/head_$rep.json 2>> $O/ont.err
done
