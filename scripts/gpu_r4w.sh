#!/bin/bash
# round 4, call r4w: the final tree -- the GPU suite, smoke, the default bench
# (every leg), then the gzip legs again with the reader's copy on one thread
# (SA_GZ_COPY_THREADS=1) for the A/B of the split copy.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r4w}
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 660 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
SA_GZ_COPY_THREADS=1 step bench_copy1 timeout -k 10 500 python -u bench.py --steps 8 --ont-leg 0 --hash-leg 0 --text-leg 0 --decode-check 0 > $O/bench_copy1.json 2> $O/bench_copy1.err
