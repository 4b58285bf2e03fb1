#!/bin/bash
# round 6, call r6l: where the command line's per-context cycle goes.  The
# 42.8 GB run (12 batches, 5 contexts) under the kernel trace with
# whole-batch staging (SA_CLI_STREAM=0, the default) and streamed staging
# (1), front_cycle.py over each, plus the wall clock of each without the
# profiler (-v stage lines kept).  First the bucket replay's per-wave probe
# (SA_BKT_PROBE): one context alone, then five; the ONT lossy batch with the
# wave-per-read prep pass (default for long reads) against 16-lane rows
# (SA_PREP_ROW=16).  The GPU suite first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6l}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E /dev/shm/sa_ont_inputs' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
INO=/dev/shm/sa_ont_inputs
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
for rep in 1 2; do
    for pr in 64 16; do
        step ont_${pr}_$rep env SA_PREP_ROW=$pr timeout -k 10 300 python -u bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/ont_${pr}_$rep.json 2>> $O/ont.err
    done
done
rm -rf $INO
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step probe_solo env SA_BKT_PROBE=$O/bkt_probe_solo.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 > $O/probe_solo.json 2> $O/probe.err
step probe_5 env SA_BKT_PROBE=$O/bkt_probe_5.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 10 > $O/probe_5.json 2>> $O/probe.err
for f in solo 5; do
    python3 scripts/bkt_probe.py $O/bkt_probe_$f.txt > $O/bkt_probe_$f.summary.txt 2>&1
    head -c 4000000 $O/bkt_probe_$f.txt | gzip -c > $O/bkt_probe_$f.head.txt.gz
    rm -f $O/bkt_probe_$f.txt
done
mkdir -p $E/l
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name stream
    local name=$1 st=$2
    sleep 3
    local t0=$(date +%s.%N)
    (cd $E/l && SA_CLI_STREAM=$st timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    local m=none
    [ $rc -eq 0 ] && m=$(md5sum $E/l/e2e.arc | cut -c1-32)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s md5 $m" >> $O/walls.txt
    rm -f $E/l/e2e.arc
    return $rc
}
cliprof() {   # name stream
    local name=$1 st=$2
    cd $E/l
    SA_CLI_STREAM=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --release > $O/cliprof_$name.log 2>&1
    local rc=$?
    rm -f e2e.arc
    cd $R
    local T=$(find $O/prof_$name -name '*kernel_trace.csv' | head -1)
    python3 scripts/front_cycle.py $T > $O/front_cycle_$name.txt 2>&1
    python3 scripts/kstats_csv.py $(find $O/prof_$name -name '*kernel_stats.csv' | head -1) > $O/kstats_$name.txt 2>&1
    rm -f $T
    find $O/prof_$name -name '*.csv' -size +2M -delete
    return $rc
}
du -sh $O >> $O/steps.txt
step cli_s0 cli s0 0
step cli_s1 cli s1 1
step prof_s0 cliprof s0 0
step prof_s1 cliprof s1 1
