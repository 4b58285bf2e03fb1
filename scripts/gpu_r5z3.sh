#!/bin/bash
# round 5, call r5z3: seqarc_amd -c --keep-clock 1 / 0 on the final tree
# (does the clock keeper still pay with the output pool?)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5z3}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1 || exit 1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir keep_clock
    local name=$1 d=$2 k=$3
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --keep-clock $k --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    cli long_k1_$rep $E/l 1 && cli long_k0_$rep $E/l 0 && cli short_k1_$rep $E/s 1 && cli short_k0_$rep $E/s 0 || exit 1
done
