#!/bin/bash
# round 4, call r4z5: the ONT-shape workload (configs[4]: SE 10-50 kbp, -l 1.15)
# with the pass-R step's v_readlane per step (SA_RV_VARIANT=0) and batched
# eight steps at a time (5, the default): 0 / 5 / 0 / 5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4z5}
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
B="bench.py --ont --pairs 60000 --lossy 1.15 --no-legs --text-leg 0 --no-verify --steps 10"
SA_RV_VARIANT=0 step ont_v0a timeout -k 10 300 python -u $B > $O/ont_v0a.json 2> $O/ont_v0a.err
step ont_v5a timeout -k 10 300 python -u $B > $O/ont_v5a.json 2> $O/ont_v5a.err
SA_RV_VARIANT=0 step ont_v0b timeout -k 10 300 python -u $B > $O/ont_v0b.json 2> $O/ont_v0b.err
step ont_v5b timeout -k 10 300 python -u $B > $O/ont_v5b.json 2> $O/ont_v5b.err
