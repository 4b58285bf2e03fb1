#!/bin/bash
# round 5, call r5f: the command line's host side and clock.
#  (0) chain_probe: cycles per pass-R step in the VALU (k_coder_rl) and on the scalar unit;
#  (1) exit_probe: process teardown time against device / page-locked memory held;
#  (2) seqarc_amd -c on the 17.8 GB (5 batches) and 42.8 GB (12 batches) files,
#      KFD's per-process eviction time (kfd_sample.py), amd-smi's throttle record
#      and the pass-R probe beside each run; host-memory variants of the long run:
#      default (registered + THP hint), SA_HOST_THP=0, SA_HOST_MALLOC=1;
#  (3) --ingest-only --devices 8 on the 42.8 GB files with 8 / 12 / 16 read threads.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5f}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $KS $SMI 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 10 amd-smi metric -g 0 -v -c -p --json >> $1 2>&1
        sleep 0.3
    done
}
step chain_probe timeout -k 10 60 scripts/bin/chain_probe > $O/chain_probe.txt 2>&1
step exit_probe timeout -k 10 240 scripts/bin/exit_probe 0 50 100 200 > $O/exit_probe.txt 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cli() {   # name dir [env...]
    local name=$1 d=$2; shift 2
    sleep 3
    python3 scripts/kfd_sample.py $O/kfd_$name.txt seqarc_amd & KS=$!
    sampler $O/smi_$name.txt & SMI=$!
    local t0=$(date +%s.%N)
    (cd $d && env "$@" SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    sleep 1
    kill $KS $SMI; wait $KS $SMI 2>/dev/null
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s X=1 && cli short_noearly $E/s SA_CLI_EARLY_READ=0 && cli short_ring4 $E/s SA_CLI_RING_SEGS=4 && cli short_ring6 $E/s SA_CLI_RING_SEGS=6 && cli short_lanes $E/s SA_RV_LANES=1 && cli long $E/l X=1 && cli long_lanes $E/l SA_RV_LANES=1 && cli long_nothp $E/l SA_HOST_THP=0 && cli long_hostmalloc $E/l SA_HOST_MALLOC=1 && cli short2 $E/s X=1 || exit 1
for t in 8 12 16; do
    (cd $E/l && timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o ing --contexts 5 --batch 69 \
        --block-size 50 --ingest-only --devices 8 --read-threads $t) > $O/ingest_$t.log 2>&1
    echo "ingest_$t rc=$?" >> $O/steps.txt
done
python3 scripts/smi_throttle.py $O/smi_*.txt > $O/throttle_report.txt 2>&1
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
