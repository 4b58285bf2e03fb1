#!/bin/bash
# round 6, call r6y: the SE / ONT / HASH legs each in a process of their own
# (bench.py --legs-fresh 1, the default now) -- the ONT leg after the headline,
# twice, then the SE and HASH legs once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6y}
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
L="--steps 2 --warmup 1 --text-leg 0 --e2e-batches 0 --ingest-devices 0 --cpu-seconds 0"
step ont_1 timeout -k 10 600 python -u bench.py $L --se-leg 0 --hash-leg 0 > $O/ont_1.json 2>> $O/err.log
step ont_2 timeout -k 10 600 python -u bench.py $L --se-leg 0 --hash-leg 0 > $O/ont_2.json 2>> $O/err.log
step all_legs timeout -k 10 900 python -u bench.py $L > $O/all_legs.json 2>> $O/err.log
