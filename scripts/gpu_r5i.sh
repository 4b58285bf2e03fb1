#!/bin/bash
# round 5, call r5i: the GPU suite on the defaults (front reads from a counter,
# the full SEQ sort), the bucket replay with its halving groups in parallel
# A/B (SA_SEQ_BUCKET=0/1, twice), then the command line's host side
# (scripts/gpu_r5f.sh as TAG r5i_cli).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5i}
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
    for bk in 0 1; do
        SA_SEQ_BUCKET=$bk step ab_b$bk timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_b${bk}_$rep.json 2>> $O/ab.err
        echo "{\"bucket\": $bk, \"rep\": $rep, \"line\": $(cat $O/ab_b${bk}_$rep.json)}" >> $O/ab_all.jsonl
    done
done
SA_SEQ_BUCKET=1 step bkt_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bkt_prof -o bkt -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/bkt.json 2> $O/bkt.err
rm -rf $IN
TAG=r5i_cli step cli bash scripts/gpu_r5f.sh
