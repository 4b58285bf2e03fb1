#!/bin/bash
# round 4, call r4k: the L passes with full-line record chunks and the
# 16-maps-per-thread L2 scan (parity suite), then the bench at 5 / 6 / 5
# contexts on the same inputs (r4c's trace: the front idles 26 % of the time
# waiting for contexts to come back from their tails).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4k}
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
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
for c in 5 6 5; do
    step bench_c$c timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --contexts $c > $O/bench_c$c.json 2> $O/bench_c$c.err
    mv $O/bench_c$c.json $O/bench_c${c}_$(date +%s).json
done
