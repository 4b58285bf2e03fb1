#!/bin/bash
# round 4, call r4d: the GPU suite (the row-cooperative aligner), then the
# pass-R probe (SA_RV_PROBE: per-wave timing, shader clock, CU / SIMD) in the
# in-HBM bench and in the CLI over the same batches, and a short bench with the
# HASH leg.  Steps as in gpu_r4c.sh (an ordinary failure does not end the call).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4d}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN /dev/shm/sa_cli_probe' EXIT
step() {
    local name=$1; shift
    "$@"; local rc=$?
    echo "$name rc=$rc" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc ${PYTEST_ARGS} > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
SA_RV_PROBE=$O/probe_bench.txt step probe_bench timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 12 > $O/probe_bench.json 2> $O/probe_bench.err
mkdir -p /dev/shm/sa_cli_probe
for m in 1 2; do for k in 1 2 3; do cat $IN/b0_r$m.fq $IN/b1_r$m.fq $IN/b2_r$m.fq $IN/b3_r$m.fq >> /dev/shm/sa_cli_probe/r$m.fq; done; done
rm -rf $IN
sleep 8
SA_RV_PROBE=$O/probe_cli.txt step probe_cli timeout -k 10 300 fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 /dev/shm/sa_cli_probe/r1.fq -2 /dev/shm/sa_cli_probe/r2.fq -o /dev/shm/sa_cli_probe/e2e --contexts 5 --batch 69 > $O/probe_cli.log 2>&1
rm -rf /dev/shm/sa_cli_probe
python3 scripts/rv_probe.py $O/probe_bench.txt $O/probe_cli.txt > $O/probe_report.txt 2>&1
step bench_hash timeout -k 10 600 python -u bench.py --batches 1 --steps 6 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --ont-leg 0 > $O/bench_hash.json 2> $O/bench_hash.err
