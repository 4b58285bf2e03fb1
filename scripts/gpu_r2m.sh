#!/bin/bash
# round 2, call m: pinned mailbox for the run's small copies -- GPU tests, H2D probe, traced e2e,
# chain priority off at C=5, kernel trace at C=1 (uncontended kernel times)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2m
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/probe_h2d.py > $O/probe_h2d.txt 2>&1 || exit 2
SA_TRACE=1 timeout -k 10 900 python -u bench.py --contexts 5 --cpu-seconds 0 --e2e-log $O/e2e_trace.log > $O/c5.json 2> $O/c5.err || exit 3
SA_CHAIN_PRIO=0 timeout -k 10 600 python -u bench.py --contexts 5 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/c5_prio0.json 2> $O/c5_prio0.err || exit 4
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 -u bench.py --contexts 1 --steps 3 --warmup 1 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/prof1_bench.json 2> $O/prof1_bench.err || exit 5
