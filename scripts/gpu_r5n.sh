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
# seqarc_amd -c --stage-ahead (each context stages its next batch into a second
# input while it encodes; round 3 measured it slower) against the default
E=/dev/shm/sa_cli_e2e
trap 'rm -rf $IN $E' EXIT
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir [seqarc_amd options...]
    local name=$1 d=$2; shift 2
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s && cli short_ahead $E/s --stage-ahead && cli long $E/l && cli long_ahead $E/l --stage-ahead \
    && SA_RV_LANES=1 cli long_lanes $E/l || exit 1
