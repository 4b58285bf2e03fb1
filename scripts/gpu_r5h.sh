#!/bin/bash
# round 5, call r5h: the front kernels' reads from a counter (k_prep_sq16 /
# k_emit_sq16, SA_FRONT_STATIC=0/1) and the bucket replay without flat LDS
# accesses (SA_SEQ_BUCKET=0/1): the GPU suite, same-call A/B of the in-HBM
# bench (no legs), twice; one context alone and five under the kernel trace;
# the ONT-shape -l 1.15 batch under the kernel trace (R-Block kernels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5h}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
INO=/dev/shm/sa_ont_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $INO' EXIT
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
    for fb in "1 0" "0 0" "1 1" "0 1"; do
        set -- $fb
        SA_FRONT_STATIC=$1 SA_SEQ_BUCKET=$2 step ab_s$1_b$2 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_s$1_b$2_$rep.json 2>> $O/ab.err
        echo "{\"static\": $1, \"bucket\": $2, \"rep\": $rep, \"line\": $(cat $O/ab_s$1_b$2_$rep.json)}" >> $O/ab_all.jsonl
    done
done
step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
step load_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/load_prof -o load -- python3 -u bench.py --inputs $IN --no-legs --no-verify --steps 16 --warmup 2 > $O/load.json 2> $O/load.err
rm -rf $IN
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 1 > $O/write_ont.log 2>&1
step ont_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ont_prof -o ont -- python3 -u bench.py --inputs $INO --ont --lossy 1.15 --batches 1 --no-legs --steps 6 --warmup 1 > $O/ont.json 2> $O/ont.err
