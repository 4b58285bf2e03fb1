#!/bin/bash
# round 5, call r5z: the kernel trace of seqarc_amd -c on the 42.8 GB files
# with the final tree (output pool, smaller ring; --keep-clock 0 under the
# profiler, --release so the trace is written at teardown) and its
# per-context cycle (front_cycle.py), against r5p's trace of the round-5 start.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r5z}
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1 || exit 1
mkdir -p $E/l
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
cd $E/l
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cliprof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --keep-clock 0 --release > $O/cli_prof.log 2>&1 || exit 5
rm -f e2e.arc
cd $R
K2=$(find $O/cliprof -name '*kernel_stats.csv' | head -1)
T2=$(find $O/cliprof -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats_csv.py $K2 > $O/cli_kernel_stats.txt 2>&1 || true
python3 scripts/front_cycle.py $T2 > $O/cli_front_cycle.txt 2>&1 || true
rm -f $T2
true
