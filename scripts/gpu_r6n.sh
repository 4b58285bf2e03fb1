#!/bin/bash
# round 6, call r6n: the command line's reader ahead by one batch (default)
# or two (SA_CLI_AHEAD_BATCHES=2: r6l showed the contexts waiting 0.15-0.28 s
# per batch for the reader, whose ring is one batch ahead), and the streamed
# staging with the whole-batch staging's 24 hardware queues (SA_CLI_HWQ=4) or
# without the helper's prefetch (SA_CLI_PREFETCH=0); 42.8 GB (long) and
# 17.8 GB (short), archives compared by MD5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6n}
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
cli() {   # name dir env...
    local name=$1 d=$2; shift 2
    sleep 3
    local t0=$(date +%s.%N)
    (cd $d && env "$@" timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    local m=none
    [ $rc -eq 0 ] && m=$(md5sum $d/e2e.arc | cut -c1-32)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s md5 $m $(grep -o 'input read [0-9.]* s\|last encode done [0-9.]* s\|reader: fill [0-9.]* s' $O/cli_$name.log | tr '\n' ' ')" >> $O/walls.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    step l_a1_$rep cli l_a1_$rep $E/l SA_CLI_AHEAD_BATCHES=1
    step l_a2_$rep cli l_a2_$rep $E/l SA_CLI_AHEAD_BATCHES=2
    step l_s1q4_$rep cli l_s1q4_$rep $E/l SA_CLI_STREAM=1 SA_CLI_HWQ=4
    step l_s1npf_$rep cli l_s1npf_$rep $E/l SA_CLI_STREAM=1 SA_CLI_PREFETCH=0
    step s_a1_$rep cli s_a1_$rep $E/s SA_CLI_AHEAD_BATCHES=1
    step s_a2_$rep cli s_a2_$rep $E/s SA_CLI_AHEAD_BATCHES=2
    step s_s1q4_$rep cli s_s1q4_$rep $E/s SA_CLI_STREAM=1 SA_CLI_HWQ=4
done
