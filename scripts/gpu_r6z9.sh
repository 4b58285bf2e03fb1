#!/bin/bash
# round 6, call r6z9: the lossy / long-read / golden GPU tests with the
# counter-fed R-Block speculative pass as the default (SA_RB_SPEC_WG=2), then
# the ONT leg as the bench runs it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z9}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "rblock or ont or lossy or golden or long or prep_row or read_counter or cli" > $O/tests.log 2>&1
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step ont_leg timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --text-leg 0 --e2e-batches 0 --ingest-devices 0 --cpu-seconds 0 --se-leg 0 --hash-leg 0 > $O/ont_leg.json 2> $O/ont_leg.err
