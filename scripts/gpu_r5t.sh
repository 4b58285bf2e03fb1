#!/bin/bash
# round 5, call r5t: the committed tree once more (after the R-Block revert):
# the GPU suite, smoke, and the ONT-shape lossy batch alone (bench.py --ont).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5t}
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
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
step ont timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont.json 2> $O/ont.err
