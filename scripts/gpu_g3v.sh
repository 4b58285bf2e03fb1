#!/bin/bash
# round 3, call g3v: grid-stride sort scatter with the next tile's keys prefetched: parity, then bench A/B
# against round 2's one-tile-per-workgroup kernel (SA_SCATTER_GRID=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3v
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py tests/test_gpu_hash.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/gs.json 2> $O/gs.err || exit 2
SA_SCATTER_GRID=1 timeout -k 10 300 $B > $O/one.json 2> $O/one.err || exit 3
timeout -k 10 300 $B > $O/gs2.json 2> $O/gs2.err || exit 4
SA_SCATTER_GRID=1 timeout -k 10 300 $B > $O/one2.json 2> $O/one2.err || exit 5
SA_SCATTER_GRID=2048 timeout -k 10 300 $B > $O/gs2048.json 2> $O/gs2048.err || exit 6
