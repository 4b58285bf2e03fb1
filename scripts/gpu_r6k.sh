#!/bin/bash
# round 6, call r6k: the bucket replay with one store per step and every step
# run (exact vmcnt waits, no wait on the last steps' stores): the GPU suite,
# the in-HBM bench twice, then one context alone under the kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6k}
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
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    step ab_$rep timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_$rep.json 2>> $O/ab.err
done
step bench_solo timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_solo -o b -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 6 > $O/bench_solo.json 2> $O/bench_solo.err
