#!/bin/bash
# round 5, call r5x: is the command line's device pipeline slowed by host
# memory being unmapped while it runs?  seqarc_amd -c on the 17.8 GB / 42.8 GB
# files: default (output buffers pooled, ring released once staged), output
# buffers fresh per block (SA_CLI_OUT_POOL=0), the ring left to the exit
# (SA_CLI_RING_FREE=0); the pass-R probe beside every run; twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5x}
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
cli() {   # name dir env
    local name=$1 d=$2 ev=$3
    sleep 8
    local t0=$(date +%s.%N)
    (cd $d && env $ev SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    cli long_$rep $E/l X=1 && cli long_nopool_$rep $E/l SA_CLI_OUT_POOL=0 && cli long_nofree_$rep $E/l SA_CLI_RING_FREE=0 \
        && cli short_$rep $E/s X=1 && cli short_nopool_$rep $E/s SA_CLI_OUT_POOL=0 && cli short_nofree_$rep $E/s SA_CLI_RING_FREE=0 || exit 1
done
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
