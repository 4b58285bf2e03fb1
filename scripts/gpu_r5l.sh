#!/bin/bash
# round 5, call r5l: the GPU suite with the bucket replay as the default; then
# seqarc_amd -c on the 17.8 GB / 42.8 GB files beside a second process keeping
# the GPU's activity up with waves that issue nothing (scripts/micro/keeper.hip
# mode 1: s_sleep) or short FMA bursts (mode 2) -- r5k's FMA keeper held the
# clock but delayed pass R's moves on the SIMDs it shared -- and with six
# contexts; amd-smi's throttle record and the pass-R probe beside every run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5l}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $SMI $KP 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
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
cli() {   # name dir keeper_mode(-: none) [seqarc_amd options...]
    local name=$1 d=$2 km=$3; shift 3
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    KP=
    if [ "$km" != - ]; then timeout -k 5 40 scripts/bin/keeper 20 1 2000 $km > $O/keeper_$name.txt 2>&1 & KP=$!; sleep 1; fi
    local t0=$(date +%s.%N)
    (cd $d && SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    if [ -n "$KP" ]; then kill $KP 2>/dev/null; wait $KP 2>/dev/null; fi
    kill $SMI; wait $SMI 2>/dev/null
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s - --contexts 5 && cli short_sleep $E/s 1 --contexts 5 && cli short_burst $E/s 2 --contexts 5 \
    && cli short_c6 $E/s - --contexts 6 && cli long $E/l - --contexts 5 && cli long_sleep $E/l 1 --contexts 5 \
    && cli long_burst $E/l 2 --contexts 5 && cli long_c6 $E/l - --contexts 6 && cli long_again $E/l - --contexts 5 || exit 1
python3 scripts/smi_throttle.py $O/smi_*.txt > $O/throttle_report.txt 2>&1
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
