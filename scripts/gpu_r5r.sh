#!/bin/bash
# round 5, call r5r: validation of the round-5 tree -- the GPU suite, smoke,
# the default bench with every leg; then the ONT-shape lossy batch (-l 1.15)
# under the kernel trace (the R-Block walks with 64-byte steps).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5r}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO /dev/shm/seqarc_bench_*' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 1 > $O/write_ont.log 2>&1
cd /tmp
step ont_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ont_prof -o ont -- python3 -u $R/bench.py --inputs $INO --ont --lossy 1.15 --batches 1 --no-legs --steps 6 --warmup 1 > $O/ont.json 2> $O/ont.err
cd $R
K=$(find $O/ont_prof -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats_csv.py $K > $O/ont_kernel_stats.txt 2>&1 || true
rm -f $(find $O/ont_prof -name '*kernel_trace.csv')
true
