#!/bin/bash
# round 3, call g4j: page-locked text windows from 2 MiB-aligned registered memory (sa_host_alloc),
# pinned by a prefill thread beside the contexts' creation; the end-to-end legs (GPU parity of the
# device parse through the stage-text tests first)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4j
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "stage_text or cli" \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 8 --cpu-seconds 0 --no-verify --e2e-log $O/e2e.log \
    > $O/bench_e2e.json 2> $O/bench_e2e.err || exit 2
