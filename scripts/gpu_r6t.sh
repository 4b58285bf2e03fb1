#!/bin/bash
# round 6, call r6t: 16 reader threads by default (r6s: the whole-node ingest
# 34-36 against 18-29 GB/s with 8) -- the command line on 42.8 GB and 17.8 GB
# with 16 against 8 (--read-threads 8), and the ingest once more.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6t}
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
cli() {   # name dir extra-args...
    local name=$1 d=$2; shift 2
    sleep 3
    local t0=$(date +%s.%N)
    (cd $d && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    local m=none
    [ $rc -eq 0 ] && [ -f $d/e2e.arc ] && m=$(md5sum $d/e2e.arc | cut -c1-32)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s md5 $m $(grep -o 'input read [0-9.]* s\|last encode done [0-9.]* s\|, [0-9.]* s, [0-9.]* MB/s' $O/cli_$name.log | tr '\n' ' ')" >> $O/walls.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    step l_t16_$rep cli l_t16_$rep $E/l
    step l_t8_$rep cli l_t8_$rep $E/l --read-threads 8
    step s_t16_$rep cli s_t16_$rep $E/s
    step s_t8_$rep cli s_t8_$rep $E/s --read-threads 8
    step i_t16_$rep cli i_t16_$rep $E/l --devices 8 --ingest-only
done
