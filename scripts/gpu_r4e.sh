#!/bin/bash
# round 4, call r4e: why pass R runs slower in the CLI than in the bench (the
# r4d probe: shader clock 2380 MHz in the bench, falling to ~1700 in the CLI).
# rocm-smi samples (power, clocks, temperature) beside each run; the probe in
#   a) the CLI (device parse), b) the CLI --host-parse, c) the in-HBM bench
#   alone, d) the in-HBM bench with a host->device copy load beside it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4e}
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
sampler() {   # sampler FILE: rocm-smi every 0.5 s until killed
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 5 rocm-smi --showpower --showclocks --showtemp --csv >> $1 2>&1
        sleep 0.5
    done
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $C
for m in 1 2; do for k in 1 2 3; do cat $IN/b0_r$m.fq $IN/b1_r$m.fq $IN/b2_r$m.fq $IN/b3_r$m.fq >> $C/r$m.fq; done; done
run_smi() {   # run_smi NAME CMD...: the sampler beside one run
    local name=$1; shift
    sampler $O/smi_$name.txt & SMI=$!
    step $name "$@"
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    sleep 8
}
CLI="fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $C/r1.fq -2 $C/r2.fq -o $C/e2e --contexts 5 --batch 69"
SA_RV_PROBE=$O/probe_cli.txt run_smi cli timeout -k 10 300 $CLI > $O/cli.log 2>&1
SA_RV_PROBE=$O/probe_cli_hostparse.txt run_smi cli_hostparse timeout -k 10 300 $CLI --host-parse > $O/cli_hostparse.log 2>&1
rm -rf $C
B="bench.py --inputs $IN --no-legs --no-verify --steps 24"
SA_RV_PROBE=$O/probe_bench.txt run_smi bench timeout -k 10 300 python -u $B > $O/bench.json 2> $O/bench.err
python -u scripts/h2d_stress.py --gbs 10 --seconds 40 > $O/h2d_stress.log 2>&1 & H2D=$!
SA_RV_PROBE=$O/probe_bench_h2d.txt run_smi bench_h2d timeout -k 10 300 python -u $B > $O/bench_h2d.json 2> $O/bench_h2d.err
wait $H2D
python3 scripts/rv_probe.py $O/probe_cli.txt $O/probe_cli_hostparse.txt $O/probe_bench.txt $O/probe_bench_h2d.txt > $O/probe_report.txt 2>&1
