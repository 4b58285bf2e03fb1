#!/bin/bash
# round 6, call r6h: the SEQ bucket replay's records stored in sorted order and
# gathered back to stream order through the bucket pass's inverse permutation
# (SA_SEQ_INV=1, k_seq_unpermute) against the scattered stores (SA_SEQ_INV=0):
# the whole GPU suite, the in-HBM bench alternating 1 / 0 twice, then the
# default bench once under the kernel trace (csv stats).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6h}
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
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    for inv in 1 0; do
        step ab_${inv}_$rep env SA_SEQ_INV=$inv timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_${inv}_$rep.json 2>> $O/ab.err
    done
done
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 -u bench.py --inputs $IN --no-legs --no-verify --steps 6 > $O/prof.json 2> $O/prof.err
