#!/bin/bash
# round 4, call r4f: the pass-R clock drop of the CLI (r4d / r4e: shader clock
# 2380 MHz in the bench, 1300-2000 in the CLI at lower board power; a
# host->device copy load did not lower it).  The in-HBM bench beside a host
# memory-copy load and beside a host arithmetic load, with rocm-smi samples and
# the pass-R probe; then the CLI once more with its reader's fill measured.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4f}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN; kill $SMI 2>/dev/null' EXIT
step() {
    local name=$1; shift
    "$@"; local rc=$?
    echo "$name rc=$rc" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 5 rocm-smi --showpower --showclocks --showtemp --csv >> $1 2>&1
        sleep 0.5
    done
}
run_smi() {
    local name=$1; shift
    sampler $O/smi_$name.txt & SMI=$!
    step $name "$@"
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    sleep 8
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
B="bench.py --inputs $IN --no-legs --no-verify --steps 32"
python -u scripts/cpu_stress.py --mode mem --threads 16 --seconds 45 > $O/stress_mem.log 2>&1 & S=$!
SA_RV_PROBE=$O/probe_bench_mem.txt run_smi bench_mem timeout -k 10 300 python -u $B > $O/bench_mem.json 2> $O/bench_mem.err
wait $S
python -u scripts/cpu_stress.py --mode alu --threads 16 --seconds 45 > $O/stress_alu.log 2>&1 & S=$!
SA_RV_PROBE=$O/probe_bench_alu.txt run_smi bench_alu timeout -k 10 300 python -u $B > $O/bench_alu.json 2> $O/bench_alu.err
wait $S
python3 scripts/rv_probe.py $O/probe_bench_mem.txt $O/probe_bench_alu.txt > $O/probe_report.txt 2>&1
