#!/bin/bash
# round 4, call r4z: what the three v_readlane per step cost pass R -- the
# diagnostic step without them (SA_RV_VARIANT=3: wrong output, the chain's
# timing only; per-wave pass-R probe) against the committed step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
SA_RV_PROBE=$O/probe_v0.txt step bench_v0 timeout -k 10 200 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 8 > $O/bench_v0.json 2> $O/bench_v0.err
SA_RV_VARIANT=3 SA_RV_PROBE=$O/probe_v3.txt step bench_v3 timeout -k 10 200 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 8 > $O/bench_v3.json 2> $O/bench_v3.err
python3 scripts/rv_probe.py $O/probe_v0.txt $O/probe_v3.txt > $O/probe_report.txt 2>&1
