#!/bin/bash
# round 5, call r5e: (1) the default bench with every leg on the previous
# SEQ path (SA_SEQ_BUCKET=0: the full sort and k_replay_seq), KFD's per-process
# eviction time sampled beside it (scripts/kfd_sample.py); (2) the GPU suite and
# smoke with the SEQ bucket replay (k_replay_seq_bkt: one sort pass over the
# context's top bits, the models of a bucket in LDS); (3) same-call A/B of the
# in-HBM bench, SA_SEQ_BUCKET=0 / 1 / 0 / 1 (no legs); (4) one context alone
# under the kernel trace (the front kernels' own times).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5e}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN /dev/shm/sa_cli_e2e; kill $KS 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
python3 scripts/kfd_sample.py $O/kfd_bench.txt & KS=$!
SA_SEQ_BUCKET=0 step bench timeout -k 10 540 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
kill $KS
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step smoke timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for v in 0 1 0 1; do
    SA_SEQ_BUCKET=$v step ab_$v timeout -k 10 300 python -u bench.py --inputs $IN --no-legs > $O/ab_$v.json 2>> $O/ab.err
    cat $O/ab_$v.json >> $O/ab_all.jsonl
done
step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
