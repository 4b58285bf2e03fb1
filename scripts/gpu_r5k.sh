#!/bin/bash
# round 5, call r5k: pass R in lanes with the pipelined feeder (k_coder_rl,
# SA_RV_LANES=1).  The GPU suite with SA_RV_LANES=1; same-call A/B of the
# in-HBM bench: lanes 0 / 1 at 5 contexts, lanes 1 at 6 contexts, the bucket
# replay by the context's low bits, twice; one
# context alone with lanes under the kernel trace.  Then seqarc_amd -c on the
# 17.8 GB / 42.8 GB files: the archive writer's threads (--writers 8 / 1) and a
# second process keeping a light VALU load on every CU (scripts/micro/keeper.hip)
# beside the tail-only phases; amd-smi's throttle record beside every run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5k}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
E=/dev/shm/sa_cli_e2e
trap 'rm -rf $IN $E; kill $KS $SMI $KP 2>/dev/null' EXIT
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
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 10 amd-smi metric -g 0 -v -c -p --json >> $1 2>&1
        sleep 0.3
    done
}
cli() {   # name dir keeper_waves_per_cu(0: none) writers
    local name=$1 d=$2 kw=$3 w=$4
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    KP=
    if [ "$kw" != 0 ]; then timeout -k 5 40 scripts/bin/keeper 20 $kw 2000 > $O/keeper_$name.txt 2>&1 & KP=$!; sleep 1; fi
    local t0=$(date +%s.%N)
    (cd $d && SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --writers $w) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    if [ -n "$KP" ]; then kill $KP 2>/dev/null; wait $KP 2>/dev/null; fi
    kill $SMI; wait $SMI 2>/dev/null
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s 0 8 && cli short_w1 $E/s 0 1 && cli short_keep1 $E/s 1 8 && cli long $E/l 0 8 && cli long_keep1 $E/l 1 8 || exit 1
python3 scripts/smi_throttle.py $O/smi_*.txt > $O/throttle_report.txt 2>&1
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
