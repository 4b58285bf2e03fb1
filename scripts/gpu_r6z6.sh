#!/bin/bash
# round 6, call r6z6: pass R's ring store issued before the segment's record
# load and three segments ahead, the slot's wait (vmcnt(5)) just before the
# group that loads it -- against the r6fin kernel (ablib/, SA_LIB): pass-R
# parity tests, the in-HBM bench interleaved, one context alone under the
# per-wave probe (shader clock, cycles per symbol).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z6}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "pass_r or coder or full_size_block or reference_test_pair or golden or many_blocks or concurrent" > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
B="bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --steps 12"
for rep in 1 2; do
    step new_$rep timeout -k 10 300 python -u $B > $O/new_$rep.json 2>> $O/ab.err
    step old_$rep env SA_LIB=$R/ablib/libseqarc_amd_r6fin.so timeout -k 10 300 python -u $B > $O/old_$rep.json 2>> $O/ab.err
done
step solo_new env SA_RV_PROBE=$O/solo_new_probe.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --contexts 1 --steps 6 > $O/solo_new.json 2> $O/solo_new.err
step solo_old env SA_LIB=$R/ablib/libseqarc_amd_r6fin.so SA_RV_PROBE=$O/solo_old_probe.txt timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --text-leg 0 --contexts 1 --steps 6 > $O/solo_old.json 2> $O/solo_old.err
python3 scripts/rv_probe.py $O/solo_new_probe.txt $O/solo_old_probe.txt > $O/report.txt 2>&1
gzip -f $O/solo_new_probe.txt $O/solo_old_probe.txt
true
