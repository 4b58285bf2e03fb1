#!/bin/bash
# round 5, call r5m: the tree with the clock keeper (seqarc_amd -c forks a
# process keeping one sleeping wave per CU resident, --keep-clock), the archive
# writer threads, the parallel page touch before pinning (SA_HOST_TOUCH) and
# the low-bit bucket replay as defaults.  (1) The GPU suite and smoke; (2) the
# default bench with every leg; (3) seqarc_amd -c on the 17.8 GB / 42.8 GB
# files: --keep-clock 1 / 0, SA_HOST_TOUCH=0, with amd-smi's throttle record
# and the pass-R probe beside every run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5m}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E /dev/shm/seqarc_bench_*; kill $SMI 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 10 amd-smi metric -g 0 -v -c -p --json >> $1 2>&1
        sleep 0.3
    done
}
cli() {   # name dir env [seqarc_amd options...]
    local name=$1 d=$2 ev=$3; shift 3
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    local t0=$(date +%s.%N)
    (cd $d && env $ev SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 "$@") > $O/cli_$name.log 2>&1
    local rc=$?
    local t1=$(date +%s.%N)
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s" >> $O/steps.txt
    kill $SMI; wait $SMI 2>/dev/null
    rm -f $d/e2e.arc
    return $rc
}
cli short $E/s X=1 && cli short_nokeep $E/s X=1 --keep-clock 0 && cli short_notouch $E/s SA_HOST_TOUCH=0 \
    && cli long $E/l X=1 && cli long_nokeep $E/l X=1 --keep-clock 0 && cli long_notouch $E/l SA_HOST_TOUCH=0 \
    && cli short2 $E/s X=1 && cli long2 $E/l X=1 || exit 1
python3 scripts/smi_throttle.py $O/smi_*.txt > $O/throttle_report.txt 2>&1
python3 scripts/rv_probe.py $O/probe_*.txt > $O/probe_report.txt 2>&1
true
