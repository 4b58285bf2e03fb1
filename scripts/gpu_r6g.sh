#!/bin/bash
# round 6, call r6g: the command line's streamed staging A/B (r6e: the reader
# faster, the device slower): old whole-batch staging / streamed / streamed with
# a hardware queue per copy stream (SA_CLI_HWQ=5) / streamed without the
# helper's prefetch of the next batch / 4 queues; 17.8 and 42.8 GB, twice.
# Then exit_probe (process teardown against VRAM and page-locked memory held).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6g}
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
    sleep 4
    local t0=$(date +%s.%N)
    (cd $d && env "$@" timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s $(grep -o 'input read [0-9.]* s\|last encode done [0-9.]* s' $O/cli_$name.log | tr '\n' ' ')" >> $O/walls.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    for leg in s l; do
        cli ${leg}_old_$rep $E/$leg SA_CLI_STREAM=0 && cli ${leg}_str_$rep $E/$leg SA_CLI_STREAM=1 && \
        cli ${leg}_str_q4_$rep $E/$leg SA_CLI_STREAM=1 SA_CLI_HWQ=4 && \
        cli ${leg}_str_nopf_$rep $E/$leg SA_CLI_STREAM=1 SA_CLI_PREFETCH=0 || exit 1
    done
done
rm -rf $E
step exit_probe timeout -k 10 240 scripts/bin/exit_probe 0 50 100 200 > $O/exit_probe.txt 2>&1
