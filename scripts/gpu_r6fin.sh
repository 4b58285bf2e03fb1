#!/bin/bash
# round 6, call r6fin: the final tree -- GPU suite, smoke, the default bench as
# the driver runs it (every leg; the CLI's -v output kept), then kernel
# statistics of the in-HBM bench under load and of one context alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6fin}
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
step tests timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step bench timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --e2e-log $O/e2e_cli.log > $O/bench.json 2> $O/bench.err
step write_inputs timeout -k 10 200 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
cd /tmp
B="$R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0"
step prof timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $B --steps 10 > $O/prof_bench.json 2> $O/prof_bench.err
step solo timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/solo -o run -- python3 -u $B --contexts 1 --steps 6 > $O/solo_bench.json 2> $O/solo_bench.err
cd $R
for d in prof solo; do
    K=$(find $O/$d -name '*kernel_stats.csv' | head -1)
    T=$(find $O/$d -name '*kernel_trace.csv' | head -1)
    python3 scripts/kstats_csv.py $K > $O/${d}_kernel_stats.txt 2>&1 || true
    python3 scripts/front_cycle.py $T > $O/${d}_front_cycle.txt 2>&1 || true
done
find $O -name '*kernel_trace.csv' -delete
find $O -name '*.csv' -size +4M -delete
true
