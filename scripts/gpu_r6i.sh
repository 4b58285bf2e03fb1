#!/bin/bash
# round 6, call r6i: (1) the R-Block chunk stride off powers of two (default
# 7904 bytes; SA_RB_CHUNK=8192 the round-5 layout), ONT lossy batch A/B;
# (2) the 10-bit SEQ bucket pass (SA_BKT_DB=10: 2^12 contexts per replay wave,
# 20 KB of LDS) against 9, in-HBM bench A/B.  The whole GPU suite first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6i}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO $IN' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
for rep in 1 2; do
    for ch in 7904 8192; do
        step ont_${ch}_$rep env SA_RB_CHUNK=$ch timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_${ch}_$rep.json 2>> $O/ont.err
    done
done
rm -rf $INO
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for db in 10 9; do
        step ab_${db}_$rep env SA_BKT_DB=$db timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_${db}_$rep.json 2>> $O/ab.err
    done
done
step prof timeout -k 10 300 env SA_BKT_DB=10 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 -u bench.py --inputs $IN --no-legs --no-verify --steps 6 > $O/prof.json 2> $O/prof.err
