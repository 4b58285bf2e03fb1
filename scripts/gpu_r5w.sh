#!/bin/bash
# round 5, call r5w: the segment ring's slots retired early.  The GPU tests of
# the command line, then --ingest-only --devices 8 on 42.8 GB and -c on the
# 17.8 GB / 42.8 GB files (each twice).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5w}
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
step cli_tests timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "cli" -o cache_dir=/tmp/pyc > $O/cli_tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir [seqarc_amd options...]
    local name=$1 d=$2; shift 2
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
cli ingest $E/l --devices 8 --ingest-only && cli ingest2 $E/l --devices 8 --ingest-only \
    && cli short $E/s && cli long $E/l && cli short2 $E/s && cli long2 $E/l || exit 1
