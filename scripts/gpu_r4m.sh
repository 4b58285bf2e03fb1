#!/bin/bash
# round 4, call r4m: does the shader clock follow the device's load?  The
# bench at a CLI-like throughput (every context pausing 1000 / 1500 ms after
# each batch) with the pass-R probe and rocm-smi; then seqarc_amd -c without
# the ramp of small first batches, and with four contexts.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4m}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $SMI 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 5 rocm-smi --showpower --showclocks --showtemp --csv >> $1 2>&1
        sleep 0.5
    done
}
cli() {   # name, extra args
    local name=$1; shift
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    (cd $E && SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    rm -f $E/e2e.arc
    echo "cli_$name rc=$rc" >> $O/steps.txt
    [ $rc -eq 0 ]
}
bgap() {   # gap ms
    sampler $O/smi_gap$1.txt & SMI=$!
    SA_RV_PROBE=$O/probe_gap$1.txt step gap$1 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 25 --step-gap-ms $1 > $O/gap$1.json 2> $O/gap$1.err
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
bgap 1500
bgap 1000
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
rm -rf $IN
cli noramp --contexts 5 --no-ramp && cli c4 --contexts 4 && cli base --contexts 5
python3 scripts/rv_probe.py $O/probe_gap1500.txt $O/probe_gap1000.txt $O/probe_noramp.txt $O/probe_c4.txt $O/probe_base.txt > $O/probe_report.txt 2>&1
