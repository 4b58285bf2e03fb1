#!/bin/bash
# round 5, call r5j: the command line's clock under its tail-only phases.
# seqarc_amd -c on the 17.8 GB and 42.8 GB files, each alone and beside a
# second process (scripts/micro/keeper.hip) that keeps a light VALU load on
# every CU (1 and 4 waves per CU); amd-smi's throttle record, KFD's eviction
# time and the pass-R probe beside every run; 8 s between runs (the bench's
# settle); then --ingest-only --devices 8 with 8 / 12 / 16 read threads.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5j}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $KS $SMI $KP 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 10 amd-smi metric -g 0 -v -c -p --json >> $1 2>&1
        sleep 0.3
    done
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir keeper_waves_per_cu(0: none) [env...]
    local name=$1 d=$2 kw=$3; shift 3
    sleep 8
    python3 scripts/kfd_sample.py $O/kfd_$name.txt seqarc_amd & KS=$!
    sampler $O/smi_$name.txt & SMI=$!
    KP=
    if [ "$kw" != 0 ]; then timeout -k 5 60 scripts/bin/keeper 25 $kw 2000 > $O/keeper_$name.txt 2>&1 & KP=$!; sleep 1; fi
    local t0=$(date +%s.%N)
    (cd $d && env "$@" SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    [ -n "$KP" ] && kill $KP 2>/dev/null; wait $KP 2>/dev/null
    sleep 1
    kill $KS $SMI; wait $KS $SMI 2>/dev/null
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s 0 X=1 && cli short_keep1 $E/s 1 X=1 && cli short_keep4 $E/s 4 X=1 && cli short_noearly $E/s 0 SA_CLI_EARLY_READ=0 \
    && cli long $E/l 0 X=1 && cli long_keep1 $E/l 1 X=1 && cli long_keep4 $E/l 4 X=1 || exit 1
for t in 8 12 16; do
    (cd $E/l && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o ing --contexts 5 --batch 69 \
        --block-size 50 --ingest-only --devices 8 --read-threads $t) > $O/ingest_$t.log 2>&1
    echo "ingest_$t rc=$?" >> $O/steps.txt
done
python3 scripts/smi_throttle.py $O/smi_*.txt > $O/throttle_report.txt 2>&1
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
