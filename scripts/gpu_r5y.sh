#!/bin/bash
# round 5, call r5y: the output-buffer pool (r5x: pass R no longer slowed by
# unmapping during the run) and the smaller segment ring.  The GPU suite, then
# seqarc_amd -c / --ingest-only with the ring at 256 MiB x 1 batch ahead
# (default) and 512 MiB x 2 batches (the round-5 start), then the default bench
# with every leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5y}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E /dev/shm/seqarc_bench_*' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir env [seqarc_amd options...]
    local name=$1 d=$2 ev=$3; shift 3
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && env $ev timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
OLD="SA_CLI_SEG_MIB=512 SA_CLI_AHEAD_BATCHES=2"
for rep in 1 2; do
    cli long_$rep $E/l X=1 && cli long_old_$rep $E/l "$OLD" && cli short_$rep $E/s X=1 && cli short_old_$rep $E/s "$OLD" \
        && cli ingest_$rep $E/l X=1 --devices 8 --ingest-only && cli ingest_old_$rep $E/l "$OLD" --devices 8 --ingest-only || exit 1
done
rm -rf $E
step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
