#!/bin/bash
# round 5, call r5s: the pass-R capacity question.  k_coder_rv holds a CU per
# workgroup of four chains (its LDS reservation), and pass R runs on st3 = the
# 3/4 of the CUs outside the long runs' set: 192 workgroups, ~4.4 batches of
# ~43.  A sixth context puts a fifth pass R in flight that cannot be placed
# (r4k: slower).  Same-call A/B of the in-HBM bench: SA_LONG_CU_EVERY = 4 / 1
# (1: every stream on every CU) x 5 / 6 contexts.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5s}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1 || exit 1
for rep in 1 2; do
    for ec in "4 5" "1 5" "1 6" "4 6"; do
        set -- $ec
        SA_LONG_CU_EVERY=$1 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --contexts $2 > $O/ab_e$1_c$2_$rep.json 2>> $O/ab.err
        rc=$?
        echo "ab_e$1_c$2 rc=$rc" >> $O/steps.txt
        [ $rc -ne 0 ] && exit $rc
        echo "{\"every\": $1, \"contexts\": $2, \"rep\": $rep, \"line\": $(cat $O/ab_e$1_c$2_$rep.json)}" >> $O/ab_all.jsonl
    done
done
