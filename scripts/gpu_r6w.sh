#!/bin/bash
# round 6, call r6w: the ONT leg's slower front -- one resident batch shared by
# the five contexts (the leg) against two (the headline runs of r6i / r6l):
# the ONT headline with one batch and with two, each in a fresh process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6w}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf /dev/shm/sa_ont1 /dev/shm/sa_ont2' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step write1 timeout -k 10 300 python -u bench.py --write-inputs /dev/shm/sa_ont1 --ont --lossy 1.15 --batches 1 > $O/write1.log 2>&1
step write2 timeout -k 10 300 python -u bench.py --write-inputs /dev/shm/sa_ont2 --ont --lossy 1.15 --batches 2 > $O/write2.log 2>&1
for rep in 1 2; do
    step one_$rep timeout -k 10 300 python -u bench.py --inputs /dev/shm/sa_ont1 --ont --lossy 1.15 --batches 1 --no-legs --steps 10 > $O/one_$rep.json 2>> $O/ont.err
    step two_$rep timeout -k 10 300 python -u bench.py --inputs /dev/shm/sa_ont2 --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/two_$rep.json 2>> $O/ont.err
done
