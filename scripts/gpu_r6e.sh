#!/bin/bash
# round 6, call r6e: the command line with streamed staging (sa_text_upload per
# block as the reader cuts it, the next batch into the other text arena while
# the current one encodes; the default) against the round-5 whole-batch staging
# (SA_CLI_STREAM=0), 17.8 GB (short) and 42.8 GB (long), twice each; first the
# streaming / staging / CLI GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6e}
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
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "text or cli" > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir stream
    local name=$1 d=$2 st=$3
    sleep 5
    local t0=$(date +%s.%N)
    (cd $d && SA_CLI_STREAM=$st timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    local m=none
    [ $rc -eq 0 ] && m=$(md5sum $d/e2e.arc | cut -c1-32)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s md5 $m" >> $O/walls.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    cli short_s1_$rep $E/s 1 && cli short_s0_$rep $E/s 0 && cli long_s1_$rep $E/l 1 && cli long_s0_$rep $E/l 0 || exit 1
done
