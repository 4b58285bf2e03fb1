#!/bin/bash
# round 4, call r4b: rocprofv3 kernel statistics and PMC traffic of the committed
# tree.  The batches are generated first, by a process that never touches the
# GPU (bench.py --write-inputs); the profiled bench only reads them (--inputs):
# no process is started inside a profiled process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r4b}
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1 || exit 1
cd /tmp
B="$R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $B --steps 10 > $O/prof_bench.json 2> $O/prof_bench.err || exit 2
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 3
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || exit 4
cd $R
F=$(find $O/pmc_fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_write -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_traffic.py $F $W $O/traffic.json > $O/traffic.txt 2>&1 || true
K=$(find $O/prof -name '*kernel_stats.csv' | head -1)
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats_csv.py $K > $O/kernel_stats.txt 2>&1 || true
python3 scripts/overlap.py $T > $O/overlap.txt 2>&1 || true
python3 scripts/front_cycle.py $T > $O/front_cycle.txt 2>&1 || true
