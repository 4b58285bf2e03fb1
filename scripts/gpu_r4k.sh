#!/bin/bash
# round 4, call r4k: (1) contexts 5 / 6 / 5 on the same inputs (r4c's trace:
# the front idles 26 % of the time waiting for contexts to come back from their
# tails), each with the staged-text leg; (2) seqarc_amd -c on the 42.8 GB files
# with the pass-R probe and rocm-smi, text windows pinned as usual and then all
# pinned before the first read (SA_CLI_PREFILL_WINDOWS): does pinning host
# memory during the run (hipHostRegister) bring the shader clock down?
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4k}
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
cli() {   # name, env...
    local name=$1; shift
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    (cd $E && env "$@" SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    rm -f $E/e2e.arc
    echo "cli_$name rc=$rc" >> $O/steps.txt
    [ $rc -eq 0 ]
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_c5a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 5 > $O/bench_c5a.json 2> $O/bench_c5a.err
step bench_c6 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 6 > $O/bench_c6.json 2> $O/bench_c6.err
step bench_c5b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 5 > $O/bench_c5b.json 2> $O/bench_c5b.err
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
rm -rf $IN
cli default && cli prepinned SA_CLI_PREFILL_WINDOWS=1100 && cli default2
python3 scripts/rv_probe.py $O/probe_default.txt $O/probe_prepinned.txt $O/probe_default2.txt > $O/probe_report.txt 2>&1
