#!/bin/bash
# round 6, call r6z5: pass R's shader clock and cycles per symbol, from the
# per-wave probe (SA_RV_PROBE: s_memtime cycles and s_memrealtime wall clock
# of every pass-R wave), one context alone and the bench's five contexts.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z5}
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
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step solo env SA_RV_PROBE=$O/solo_probe.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --contexts 1 --steps 6 > $O/solo.json 2> $O/solo.err
step loaded env SA_RV_PROBE=$O/loaded_probe.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 10 > $O/loaded.json 2> $O/loaded.err
python3 scripts/rv_probe.py $O/solo_probe.txt $O/loaded_probe.txt > $O/report.txt 2>&1
gzip -f $O/solo_probe.txt $O/loaded_probe.txt
true
