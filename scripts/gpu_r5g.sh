#!/bin/bash
# round 5, call r5g: pass R in lanes (k_coder_rl, SA_RV_LANES=1) and the SEQ
# bucket replay with its 8-step prefetch (SA_SEQ_BUCKET).  The GPU suite with
# SA_RV_LANES=1 (every context on k_coder_rl); then same-call A/B of the
# in-HBM bench over (lanes, bucket) in {0,1}^2, twice; then the kernel
# statistics of one context alone and of the default five with lanes + bucket.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5g}
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
SA_RV_LANES=1 step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for lb in "0 0" "1 0" "0 1" "1 1"; do
        set -- $lb
        SA_RV_LANES=$1 SA_SEQ_BUCKET=$2 step ab_l$1_b$2 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_l$1_b$2_$rep.json 2>> $O/ab.err
        echo "{\"lanes\": $1, \"bucket\": $2, \"rep\": $rep, \"line\": $(cat $O/ab_l$1_b$2_$rep.json)}" >> $O/ab_all.jsonl
    done
done
SA_RV_LANES=1 step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
SA_RV_LANES=1 step load_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/load_prof -o load -- python3 -u bench.py --inputs $IN --no-legs --no-verify --steps 16 --warmup 2 > $O/load.json 2> $O/load.err
