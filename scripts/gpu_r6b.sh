#!/bin/bash
# round 6, call r6b: pass R with its operands through SMEM (k_coder_rv<6>, the
# new default): the pass-R parity tests first, then the GPU suite and smoke,
# then same-call A/B of the in-HBM bench (SA_RV_VARIANT=5 / 6, twice), then
# one context alone under the kernel trace (pass R's solo time).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6b}
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
step passr timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "pass_r or coder or full_size_block or starved" > $O/passr.log 2>&1
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for v in 5 6 5 6; do
    SA_RV_VARIANT=$v step ab_$v timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_$v.json 2>> $O/ab.err
    echo "{\"variant\": $v, \"line\": $(cat $O/ab_$v.json)}" >> $O/ab_all.jsonl
done
step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
