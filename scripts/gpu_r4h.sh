#!/bin/bash
# round 4, call r4h: the CLI's pass-R clock drop (r4d-r4g: neither host memory
# traffic, host->device copies nor a bursty load lowered the bench's clock).
# The CLI sets SA_SYNC=block (host threads sleep on their streams); the bench
# spins.  CLI block / spin, bench spin / block, with the probe and rocm-smi.
# Also: the L passes on their own CUs (SA_L_CU_EVERY=4 / 2) in the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4h}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
C=/dev/shm/sa_cli_probe
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $C; kill $SMI 2>/dev/null' EXIT
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
B="bench.py --inputs $IN --no-legs --no-verify --steps 24"
SA_RV_PROBE=$O/probe_bench_block.txt SA_SYNC=block run_smi bench_block timeout -k 10 300 python -u $B > $O/bench_block.json 2> $O/bench_block.err
SA_L_CU_EVERY=4 run_smi bench_l4 timeout -k 10 300 python -u $B > $O/bench_l4.json 2> $O/bench_l4.err
SA_L_CU_EVERY=2 run_smi bench_l2 timeout -k 10 300 python -u $B > $O/bench_l2.json 2> $O/bench_l2.err
run_smi bench_base timeout -k 10 300 python -u $B > $O/bench_base.json 2> $O/bench_base.err
mkdir -p $C
for m in 1 2; do for k in 1 2 3; do cat $IN/b0_r$m.fq $IN/b1_r$m.fq $IN/b2_r$m.fq $IN/b3_r$m.fq >> $C/r$m.fq; done; done
rm -rf $IN
CLI="fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $C/r1.fq -2 $C/r2.fq -o $C/e2e --contexts 5 --batch 69"
SA_RV_PROBE=$O/probe_cli_spin.txt SA_SYNC=spin run_smi cli_spin timeout -k 10 300 $CLI > $O/cli_spin.log 2>&1
SA_RV_PROBE=$O/probe_cli_block.txt run_smi cli_block timeout -k 10 300 $CLI > $O/cli_block.log 2>&1
python3 scripts/rv_probe.py $O/probe_bench_block.txt $O/probe_cli_spin.txt $O/probe_cli_block.txt > $O/probe_report.txt 2>&1
