#!/bin/bash
# round 3, call g3m (after the container was re-created): the GPU suite in one process, the bench with
# its e2e (short + long) and gzip legs, pass-R step variant A/B (SA_RV_V2), the GRCh38-sized HASH bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3m
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 2
B="python -u bench.py --steps 12 --e2e-batches 0 --cpu-seconds 0 --no-verify"
SA_RV_V2=1 timeout -k 10 300 $B > $O/c5_v2.json 2> $O/c5_v2.err || exit 3
timeout -k 10 300 $B > $O/c5_v0.json 2> $O/c5_v0.err || exit 4
timeout -k 10 600 python -u scripts/bench_hash.py > $O/hash.json 2> $O/hash.err || exit 5
