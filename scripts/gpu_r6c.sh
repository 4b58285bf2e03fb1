#!/bin/bash
# round 6, call r6c: pass R through SMEM (V6) beside the fronts -- its chains
# hold their SIMDs' scalar issue (10 SALU per ~45 cycles), so the kernels
# sharing those SIMDs slowed (r6b: L passes 89 vs 50 ms, SEQ sort 40 vs 22).
# Same-call A/B of the in-HBM bench: V5 / V6 / V6 at chain priority 0 / V6
# with the L passes on all CUs / V6 with pass R on 5 or 4 of each 8 CUs and
# the L passes on the front's CUs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6c}
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
ab() {   # name env...
    local name=$1; shift
    step ab_$name timeout -k 10 300 env "$@" python -u bench.py --inputs $IN --no-legs > $O/ab_$name.json 2>> $O/ab.err
    echo "{\"name\": \"$name\", \"line\": $(cat $O/ab_$name.json)}" >> $O/ab_all.jsonl
}
ab v5 SA_RV_VARIANT=5
ab v6 SA_RV_VARIANT=6
ab v6_prio0 SA_RV_VARIANT=6 SA_CHAIN_PRIO=0
ab v6_lall SA_RV_VARIANT=6 SA_L_CU_EVERY=1
ab v6_cus5 SA_RV_VARIANT=6 SA_RV_CUS=5 SA_L_CU_EVERY=1
ab v6_cus4 SA_RV_VARIANT=6 SA_RV_CUS=4 SA_L_CU_EVERY=1
ab v5_cus5 SA_RV_VARIANT=5 SA_RV_CUS=5 SA_L_CU_EVERY=1
ab v5b SA_RV_VARIANT=5
ab v6b SA_RV_VARIANT=6
