#!/bin/bash
# round 6, call r6z2: the output blocks' device-to-host copies through the
# runtime's staging buffer instead of pinning the pool's pageable buffers
# (GPU_PINNED_MIN_XFER_SIZE above any block's size): the exit's teardown of the
# pinned pages (r6z: ~0.2-0.3 s of exit -> reaped) against the copies' host
# memcpy; 17.8 GB and 42.8 GB, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z2}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
S=GPU_PINNED_MIN_XFER_SIZE:4096
step short timeout -k 10 600 python3 -u scripts/cli_exit_ab.py $E/s $O/short_ab.txt \
    def1= stg1=$S def2= stg2=$S def3= stg3=$S
step long timeout -k 10 600 python3 -u scripts/cli_exit_ab.py $E/l $O/long_ab.txt \
    def1= stg1=$S def2= stg2=$S
