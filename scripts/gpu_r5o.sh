#!/bin/bash
# round 5, call r5o: k_coder_rl with the ring handed over by an LDS-only
# barrier (__syncthreads' fence waited for every outstanding global access: the
# feeders' next-round loads, the chain's checkpoint store).  Parity of both
# pass-R kernels; same-call A/B of the in-HBM bench, lanes 0 / 1 twice; the
# release cost of a 512 MiB-segment ring (pin_probe); seqarc_amd -c with the
# ring released on 8 threads (default) / 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5o}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step paths timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pass_r_and_seq or starved" -o cache_dir=/tmp/pyc > $O/paths.log 2>&1
SA_RV_LANES=1 step starved_lanes timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "starved" -o cache_dir=/tmp/pyc > $O/starved_lanes.log 2>&1
step pin_probe timeout -k 10 180 scripts/bin/pin_probe 8 > $O/pin_probe.txt 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for l in 0 1; do
        SA_RV_LANES=$l step ab_l$l timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_l${l}_$rep.json 2>> $O/ab.err
        echo "{\"lanes\": $l, \"rep\": $rep, \"line\": $(cat $O/ab_l${l}_$rep.json)}" >> $O/ab_all.jsonl
    done
done
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir env [seqarc_amd options...]
    local name=$1 d=$2 ev=$3; shift 3
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && env $ev timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s X=1 && cli short_free1 $E/s SA_CLI_FREE_THREADS=1 && cli long $E/l X=1 && cli long_free1 $E/l SA_CLI_FREE_THREADS=1 \
    && cli long_lanes $E/l SA_RV_LANES=1 || exit 1
