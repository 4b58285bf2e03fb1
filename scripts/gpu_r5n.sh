#!/bin/bash
# round 5, call r5n: pass R in lanes with coalesced feeders (k_coder_rl: four
# feeder waves load each chain's segment whole and convert it into an LDS
# ring; SA_RV_LANES=1).  The parity tests of both pass-R kernels, then the GPU
# suite with lanes, then same-call A/B of the in-HBM bench, lanes 0 / 1 twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5n}
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
step paths timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pass_r_and_seq or starved" -o cache_dir=/tmp/pyc > $O/paths.log 2>&1
SA_RV_LANES=1 step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for l in 0 1; do
        SA_RV_LANES=$l step ab_l$l timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_l${l}_$rep.json 2>> $O/ab.err
        echo "{\"lanes\": $l, \"rep\": $rep, \"line\": $(cat $O/ab_l${l}_$rep.json)}" >> $O/ab_all.jsonl
    done
done
