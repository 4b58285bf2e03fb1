#!/bin/bash
# round 6, call r6m: the bucket replay's digits largest first (k_bkt_order,
# default) against digit order (SA_BKT_LPT=0), and pass R through SMEM
# (SA_RV_VARIANT=6) on this tree, in-HBM bench alternating twice; the replay
# probe with one context; the GPU suite first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6m}
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
    step ab_lpt_$rep timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_lpt_$rep.json 2>> $O/ab.err
    step ab_nolpt_$rep env SA_BKT_LPT=0 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_nolpt_$rep.json 2>> $O/ab.err
    step ab_v6_$rep env SA_RV_VARIANT=6 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_v6_$rep.json 2>> $O/ab.err
done
step probe_solo env SA_BKT_PROBE=$O/bkt_probe_solo.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 > $O/probe_solo.json 2> $O/probe.err
python3 scripts/bkt_probe.py $O/bkt_probe_solo.txt > $O/bkt_probe_solo.summary.txt 2>&1
rm -f $O/bkt_probe_solo.txt
