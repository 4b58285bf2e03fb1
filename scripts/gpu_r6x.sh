#!/bin/bash
# round 6, call r6x: the ONT leg after the headline (a second set of contexts
# in the process) with the bench's 24 hardware queues against 32
# (SA_BENCH_HWQ): is the leg's slower front the new contexts' streams sharing
# queues?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6x}
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
L="--steps 2 --warmup 1 --text-leg 0 --se-leg 0 --hash-leg 0 --e2e-batches 0 --ingest-devices 0 --cpu-seconds 0"
for rep in 1 2; do
    step q24_$rep timeout -k 10 600 python -u bench.py $L > $O/q24_$rep.json 2>> $O/err.log
    step q32_$rep env SA_BENCH_HWQ=32 timeout -k 10 600 python -u bench.py $L > $O/q32_$rep.json 2>> $O/err.log
done
