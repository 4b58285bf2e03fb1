#!/bin/bash
# round 6, call r6j: kernel times with ONE context (no other batch's pass R
# beside the front): the ONT lossy batch and the in-HBM bench batch under the
# kernel trace, for the R-Block / prep / replay kernels' solo durations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6j}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO $IN' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
step ont_solo timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ont_solo -o o -- python3 -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --no-verify --contexts 1 --steps 6 > $O/ont_solo.json 2> $O/ont_solo.err
rm -rf $INO
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_solo timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_solo -o b -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 6 > $O/bench_solo.json 2> $O/bench_solo.err
