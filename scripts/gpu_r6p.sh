#!/bin/bash
# round 6, call r6p: the round-6 tree (pass R through SMEM by default for
# short reads, the tile-staged k_seq_unpermute): GPU suite, the in-HBM bench
# twice, then the profile set as round 5's r5p -- rocprofv3 kernel statistics
# under the bench's load and of one context alone, FETCH_SIZE / WRITE_SIZE
# passes (pmc_traffic.py -> traffic.json), the bench's front cycle, and the
# command line's kernel trace on the 42.8 GB files with its front cycle.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6p}
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
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for rep in 1 2; do
    step ab_$rep timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_$rep.json 2>> $O/ab.err
done
mkdir -p $E/l
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
cd /tmp
B="$R/bench.py --inputs $IN --no-legs --no-verify --text-leg 0"
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $B --steps 10 > $O/prof_bench.json 2> $O/prof_bench.err
step solo timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/solo -o run -- python3 -u $B --contexts 1 --steps 6 > $O/solo_bench.json 2> $O/solo_bench.err
step pmc_fetch timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err
step pmc_write timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u $B --steps 2 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err
rm -rf $IN
cd $E/l
step cliprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cliprof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 --release > $O/cli_prof.log 2>&1
rm -f e2e.arc
cd $R
F=$(find $O/pmc_fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_write -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_traffic.py $F $W $O/traffic.json > $O/traffic.txt 2>&1 || true
for d in prof solo cliprof; do
    K=$(find $O/$d -name '*kernel_stats.csv' | head -1)
    T=$(find $O/$d -name '*kernel_trace.csv' | head -1)
    python3 scripts/kstats_csv.py $K > $O/${d}_kernel_stats.txt 2>&1 || true
    python3 scripts/front_cycle.py $T > $O/${d}_front_cycle.txt 2>&1 || true
    python3 scripts/overlap.py $T > $O/${d}_overlap.txt 2>&1 || true
done
rm -f $F $W
find $O -name '*kernel_trace.csv' -delete
find $O -name '*.csv' -size +4M -delete
du -sh $O >> $O/steps.txt
true
