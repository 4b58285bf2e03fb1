#!/bin/bash
# round 4, call r4k: contexts 5 / 6 / 5 on the same inputs (r4c's trace: the
# front idles 26 % of the time waiting for contexts to come back from their
# tails), each with the staged-text leg; then one run with the pass-R probe and
# rocm-smi: are the staged-text leg's batches (H2D from registered huge-page
# memory + device parse, as in seqarc_amd -c) at the bench's shader clock?
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4k}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN; kill $SMI 2>/dev/null' EXIT
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
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step bench_c5a timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 5 > $O/bench_c5a.json 2> $O/bench_c5a.err
step bench_c6 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 6 > $O/bench_c6.json 2> $O/bench_c6.err
step bench_c5b timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 5 > $O/bench_c5b.json 2> $O/bench_c5b.err
sampler $O/smi_probe.txt & SMI=$!
SA_RV_PROBE=$O/probe.txt step bench_probe timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 15 --warmup 0 > $O/bench_probe.json 2> $O/bench_probe.err
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
python3 scripts/rv_probe.py $O/probe.txt > $O/probe_report.txt 2>&1
