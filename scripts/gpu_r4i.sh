#!/bin/bash
# round 4, call r4i: the GPU suite (dense AUX sort, branch-free emit), the
# bench at a CLI-like throughput (each context idle 1500 ms per batch: does the
# shader clock follow the load?), the default bench with every leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4i}
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
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
sampler $O/smi_gap1500.txt & SMI=$!
SA_RV_PROBE=$O/probe_gap1500.txt step gap1500 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 20 --step-gap-ms 1500 > $O/gap1500.json 2> $O/gap1500.err
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
rm -rf $IN
python3 scripts/rv_probe.py $O/probe_gap1500.txt > $O/probe_report.txt 2>&1
sleep 5
step bench timeout -k 10 1000 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
