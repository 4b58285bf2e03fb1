#!/bin/bash
# round 5, call r5d: the GPU suite and the default bench with every leg on the
# tree after the re-entry (R-Block tables, the dege read list, SWAR N-gap pass,
# the segment reader, the SE leg), KFD's per-process eviction time sampled
# beside the bench (scripts/kfd_sample.py), then the kernel statistics of one
# context alone (the front kernels' own times, no pipeline overlap).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5d}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN /dev/shm/sa_cli_e2e; kill $KS 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
python3 scripts/kfd_sample.py $O/kfd_bench.txt & KS=$!
step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
kill $KS
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
