#!/bin/bash
# round 5, call r5b: (1) the firmware's throttle record next to the clocks:
# amd-smi metric -v -c -p (violation accumulators: PPT, thermal, PROCHOT, HBM,
# per-XCD "clock below host limit" power / thermal / total and low-utilization)
# sampled through the in-HBM bench and through seqarc_amd -c on the 42.8 GB
# files, with the pass-R probe in both; (2) a kernel trace of the ONT-shape
# -l 1.15 batch (what "prep+scan" holds there).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5b}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
INO=/dev/shm/sa_ont_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $INO $E; kill $SMI 2>/dev/null' EXIT
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
        timeout 10 amd-smi metric -g 0 -v -c -p --json >> $1 2>&1
        sleep 0.3
    done
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
sleep 5
sampler $O/smi_bench.txt & SMI=$!
SA_RV_PROBE=$O/probe_bench.txt step bench timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 24 > $O/bench.json 2> $O/bench.err
kill $SMI; wait $SMI 2>/dev/null
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
rm -rf $IN
sleep 8
sampler $O/smi_cli.txt & SMI=$!
(cd $E && SA_RV_PROBE=$O/probe_cli.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
    -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli.log 2>&1
echo "cli rc=$?" >> $O/steps.txt
sleep 2
kill $SMI; wait $SMI 2>/dev/null
rm -rf $E
python3 scripts/rv_probe.py $O/probe_bench.txt $O/probe_cli.txt > $O/probe_report.txt 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 1 > $O/write_ont.log 2>&1
step ont_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ont_prof -o ont -- python3 -u bench.py --inputs $INO --ont --lossy 1.15 --batches 1 --no-legs --no-verify --steps 4 --warmup 1 > $O/ont.json 2> $O/ont.err
