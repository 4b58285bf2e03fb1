#!/bin/bash
# round 5, call r5k: pass R in lanes with the pipelined feeder (k_coder_rl,
# SA_RV_LANES=1).  The GPU suite with SA_RV_LANES=1; same-call A/B of the
# in-HBM bench: lanes 0 / 1 at 5 contexts, lanes 1 at 6 contexts, the bucket
# replay by the context's low bits, twice; one
# context alone with lanes under the kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5k}
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
step pin_probe timeout -k 10 120 scripts/bin/pin_probe 8 > $O/pin_probe.txt 2>&1
SA_RV_LANES=1 step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for lcb in "0 5 0" "1 5 0" "1 6 0" "0 5 1"; do
        set -- $lcb
        SA_RV_LANES=$1 SA_SEQ_BUCKET=$3 step ab_l$1_c$2_b$3 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --contexts $2 > $O/ab_l$1_c$2_b$3_$rep.json 2>> $O/ab.err
        echo "{\"lanes\": $1, \"contexts\": $2, \"bucket\": $3, \"rep\": $rep, \"line\": $(cat $O/ab_l$1_c$2_b$3_$rep.json)}" >> $O/ab_all.jsonl
    done
done
SA_RV_LANES=1 step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
