#!/bin/bash
# round 6, call r6o: the bucket pass with 9-bit digits at Slevel 3
# (SA_BKT_DB=9: 2^11 contexts, 10 KB of LDS per replay wave, twice the waves
# per CU) against 8, bench A/B and the replay probe; then the command line
# with pass R through SMEM (SA_RV_VARIANT=6) against the default, long and
# short.  The GPU suite first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6o}
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
    step ab_db9_$rep env SA_BKT_DB=9 timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_db9_$rep.json 2>> $O/ab.err
    step ab_db8_$rep timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_db8_$rep.json 2>> $O/ab.err
done
step probe_db9 env SA_BKT_DB=9 SA_BKT_PROBE=$O/bkt_probe_db9.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 > $O/probe_db9.json 2> $O/probe.err
python3 scripts/bkt_probe.py $O/bkt_probe_db9.txt > $O/bkt_probe_db9.summary.txt 2>&1
rm -f $O/bkt_probe_db9.txt
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
    echo "$name rc=$rc wall $(python3 -c "print(round($t1-$t0,3))") s md5 $m $(grep -o 'input read [0-9.]* s\|last encode done [0-9.]* s\|, [0-9.]* s, [0-9.]* MB/s' $O/cli_$name.log | tr '\n' ' ')" >> $O/walls.txt
    rm -f $d/e2e.arc
    return $rc
}
for rep in 1 2; do
    step l_v5_$rep cli l_v5_$rep $E/l SA_RV_VARIANT=-1
    step l_v6_$rep cli l_v6_$rep $E/l SA_RV_VARIANT=6
    step s_v5_$rep cli s_v5_$rep $E/s SA_RV_VARIANT=-1
    step s_v6_$rep cli s_v6_$rep $E/s SA_RV_VARIANT=6
done
