#!/bin/bash
# round 6, call r6f: the R-Block speculative pass without per-byte branches
# (rb_spec_vals: selects, a loop-free rounded root, every lane walking its 8 KiB
# chunk in step): the lossy GPU tests, then the ONT-shape lossy batch alone
# (bench.py --ont --lossy 1.15) twice, the in-HBM bench twice (the L passes'
# full-segment path), and the ONT batch once under the kernel trace.  The whole
# GPU suite first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6f}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO /dev/shm/sa_bench_inputs' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
for rep in 1 2; do
    step ont_$rep timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_$rep.json 2>> $O/ont.err
done
IN=/dev/shm/sa_bench_inputs
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    step ab_$rep timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_$rep.json 2>> $O/ab.err
done
rm -rf $IN
step ont_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ont_prof -o ont -- python3 -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --no-verify --steps 6 > $O/ont_prof.json 2> $O/ont_prof.err
