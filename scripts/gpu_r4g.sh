#!/bin/bash
# round 4, call r4g: is the CLI's pass-R clock drop (r4d-r4f) the bursty load?
# The in-HBM bench with each context idle 300 / 700 ms after each batch (the
# CLI's contexts wait for the reader), and the CLI with --stage-ahead; probe +
# rocm-smi samples.  Also checks the branch-free emit (GPU suite of the parity tests).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4g}
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
step parity timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/parity.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
B="bench.py --inputs $IN --no-legs --no-verify --steps 24"
SA_RV_PROBE=$O/probe_gap700.txt run_smi gap700 timeout -k 10 300 python -u $B --step-gap-ms 700 > $O/gap700.json 2> $O/gap700.err
SA_RV_PROBE=$O/probe_gap300.txt run_smi gap300 timeout -k 10 300 python -u $B --step-gap-ms 300 > $O/gap300.json 2> $O/gap300.err
mkdir -p $C
for m in 1 2; do for k in 1 2 3; do cat $IN/b0_r$m.fq $IN/b1_r$m.fq $IN/b2_r$m.fq $IN/b3_r$m.fq >> $C/r$m.fq; done; done
rm -rf $IN
CLI="fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $C/r1.fq -2 $C/r2.fq -o $C/e2e --contexts 5 --batch 69"
SA_RV_PROBE=$O/probe_cli.txt run_smi cli timeout -k 10 300 $CLI > $O/cli.log 2>&1
SA_RV_PROBE=$O/probe_cli_ahead.txt run_smi cli_ahead timeout -k 10 300 $CLI --stage-ahead > $O/cli_ahead.log 2>&1
python3 scripts/rv_probe.py $O/probe_gap700.txt $O/probe_gap300.txt $O/probe_cli.txt $O/probe_cli_ahead.txt > $O/probe_report.txt 2>&1
