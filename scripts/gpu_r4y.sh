#!/bin/bash
# round 4, call r4y: the L passes with the records staged through LDS by
# wave-wide loads (k_coder_l1s / k_coder_l3s, the default) against the
# per-lane loads (SA_L_STAGE=0): the GPU parity suite with staging, then the
# bench on / off / on on the same inputs, then one rocprofv3 kernel-trace pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4y}
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
step parity timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_sa timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_sa.json 2> $O/bench_sa.err
SA_L_STAGE=0 step bench_off timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_off.json 2> $O/bench_off.err
step bench_sb timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --text-leg 0 > $O/bench_sb.json 2> $O/bench_sb.err
cd /tmp
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 10 > $O/prof_bench.json 2> $O/prof_bench.err
cd $R
K=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats_csv.py $K > $O/kernel_stats.txt 2>&1 || true
