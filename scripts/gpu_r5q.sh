#!/bin/bash
# round 5, call r5q: same-call A/B of the in-HBM bench with pass R and the L
# passes confined to n of each 8 CUs and the front stream on the others
# (SA_RV_CUS = unset / 5 / 4), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5q}
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
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for n in 0 5 4; do
        if [ $n = 0 ]; then ev="X=1"; else ev="SA_RV_CUS=$n"; fi
        env $ev timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_c${n}_$rep.json 2>> $O/ab.err
        rc=$?
        echo "ab_c$n rc=$rc" >> $O/steps.txt
        [ $rc -ne 0 ] && exit $rc
        echo "{\"rv_cus\": $n, \"rep\": $rep, \"line\": $(cat $O/ab_c${n}_$rep.json)}" >> $O/ab_all.jsonl
    done
done
