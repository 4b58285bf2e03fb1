#!/bin/bash
# round 6, call r6z3: the R-Block entry pass a wave per block (k_rb_fix_w,
# default) against a lane per block (k_rb_fix, SA_RB_FIX_SERIAL=1): the lossy
# GPU tests, the ONT-shape lossy batch alone twice each way (interleaved), and
# the default once under the kernel trace; also the front kernels taking
# reads from the counter by the batch's mean read length (4 at a time for the ONT
# shape instead of 64).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z3}
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
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "rblock or ont or long_read or prep_row or read_counter or reference_test_pair or sub_batches" > $O/tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
for rep in 1 2; do
    step ont_w_$rep timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_w_$rep.json 2>> $O/ont.err
    step ont_s_$rep env SA_RB_FIX_SERIAL=1 timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_s_$rep.json 2>> $O/ont.err
done
cd /tmp
step ont_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ont_prof -o ont -- python3 -u $R/bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --no-verify --steps 6 > $O/ont_prof.json 2> $O/ont_prof.err
