#!/bin/bash
# round 4, call r4t: the GPU suite on the tree with the lane-parallel side-stream
# read test (k_emit_sq) and the batched AUX presence bitmap, then the default
# bench, then the profile set of scripts/gpu_r4b.sh (kernel statistics, PMC).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-legs --text-leg 0 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" >> $O/steps.txt
[ $rc -eq 0 ] || exit $rc
TAG=r4t/prof_set bash scripts/gpu_r4b.sh
