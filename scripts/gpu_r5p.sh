#!/bin/bash
# round 5, call r5p: rocprofv3 kernel statistics and PMC traffic of the
# round-5 tree (as scripts/gpu_r4b.sh: the batches written by a process that
# never touches the GPU, the profiled bench only reads them), then the kernel
# trace of seqarc_amd -c on the 42.8 GB files (--keep-clock 0: no companion
# process under the profiler; --release: the trace is written at teardown) and
# the per-context cycle of both traces (front_cycle.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r5p}
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1 || exit 1
mkdir -p $E/l
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
cd /tmp
B="$R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $B --steps 10 > $O/prof_bench.json 2> $O/prof_bench.err || exit 2
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 3
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || exit 4
rm -rf $IN
cd $E/l
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cliprof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --keep-clock 0 --release > $O/cli_prof.log 2>&1 || exit 5
rm -f e2e.arc
cd $R
F=$(find $O/pmc_fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_write -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_traffic.py $F $W $O/traffic.json > $O/traffic.txt 2>&1 || true
K=$(find $O/prof -name '*kernel_stats.csv' | head -1)
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats_csv.py $K > $O/kernel_stats.txt 2>&1 || true
python3 scripts/overlap.py $T > $O/overlap.txt 2>&1 || true
python3 scripts/front_cycle.py $T > $O/front_cycle.txt 2>&1 || true
K2=$(find $O/cliprof -name '*kernel_stats.csv' | head -1)
T2=$(find $O/cliprof -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats_csv.py $K2 > $O/cli_kernel_stats.txt 2>&1 || true
python3 scripts/front_cycle.py $T2 > $O/cli_front_cycle.txt 2>&1 || true
rm -f $T2
true
