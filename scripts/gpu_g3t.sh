#!/bin/bash
# round 3, call g3t: parity (16-bit scatter counters, word-wise name suffixes, pass R without the V2 step);
# parity and bench with pass R partitioned per context (SA_RV_PART=1); front stream priority; chain priority off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3t
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
SA_RV_PART=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "concurrent or full_size or reference_test_pair or many_blocks" > $O/parity_part.log 2>&1 || exit 2
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/base.json 2> $O/base.err || exit 3
SA_RV_PART=1 timeout -k 10 300 $B > $O/part.json 2> $O/part.err || exit 4
SA_FRONT_PRIO=1 timeout -k 10 300 $B > $O/fprio.json 2> $O/fprio.err || exit 5
SA_CHAIN_PRIO=0 timeout -k 10 300 $B > $O/prio0.json 2> $O/prio0.err || exit 6
timeout -k 10 300 $B > $O/base2.json 2> $O/base2.err || exit 7
SA_RV_PART=1 timeout -k 10 300 $B > $O/part2.json 2> $O/part2.err || exit 8
