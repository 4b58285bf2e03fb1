#!/bin/bash
# round 6, call r6s: (1) the ONT leg alone after a short headline (is the full
# bench's 61 ms of prep+scan the leg's or the run's?), (2) the whole-node
# ingest (--ingest-only --devices 8) with the reader one (default), two or
# three batches ahead and with 16 read threads, (3) the batched-move pass R
# (SA_RV_VARIANT=5) on the final tree: PMC traffic and the bench's front cycle,
# for the record beside r6r's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6s}
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
step ontleg timeout -k 10 600 python -u bench.py --steps 4 --warmup 2 --text-leg 0 --se-leg 0 --hash-leg 0 --e2e-batches 0 --ingest-devices 0 --cpu-seconds 0 > $O/ontleg.json 2> $O/ontleg.err
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/l
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
ing() {   # name env...
    local name=$1; shift
    local t0=$(date +%s.%N)
    (cd $E/l && env "$@" timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o e2e \
        --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --devices 8 --ingest-only $EXTRA) > $O/ing_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s $(grep -o 'input read [0-9.]* s\|reader: fill [0-9.]* s, cut [0-9.]* s\|, [0-9.]* s, [0-9.]* MB/s' $O/ing_$name.log | tr '\n' ' ')" >> $O/ingest.txt
    rm -f $E/l/e2e.arc
    return $rc
}
for rep in 1 2; do
    step ing_a1_$rep ing a1_$rep SA_CLI_AHEAD_BATCHES=1
    step ing_a2_$rep ing a2_$rep SA_CLI_AHEAD_BATCHES=2
    step ing_a3_$rep ing a3_$rep SA_CLI_AHEAD_BATCHES=3
    EXTRA="--read-threads 16" step ing_t16_$rep ing t16_$rep SA_CLI_AHEAD_BATCHES=1
done
rm -rf $E
cd /tmp
B="$R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0"
step prof5 env SA_RV_VARIANT=5 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o run -- python3 -u $B --steps 10 > $O/prof5_bench.json 2> $O/prof5_bench.err
step pmc5_fetch env SA_RV_VARIANT=5 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc5_fetch -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc5_fetch.json 2> $O/pmc5_fetch.err
step pmc5_write env SA_RV_VARIANT=5 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc5_write -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc5_write.json 2> $O/pmc5_write.err
cd $R
F=$(find $O/pmc5_fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc5_write -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_traffic.py $F $W $O/traffic5.json > $O/traffic5.txt 2>&1 || true
K=$(find $O/prof5 -name '*kernel_stats.csv' | head -1)
T=$(find $O/prof5 -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats_csv.py $K > $O/prof5_kernel_stats.txt 2>&1 || true
python3 scripts/front_cycle.py $T > $O/prof5_front_cycle.txt 2>&1 || true
rm -f $F $W
find $O -name '*kernel_trace.csv' -delete
find $O -name '*.csv' -size +4M -delete
true
