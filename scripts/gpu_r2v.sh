#!/bin/bash
# round 2, call v: device FASTQ parse (sa_stage_text) + pinned text windows in the CLI; MD5 pipelined LDS
# reads; GPU suite, default bench (end to end over 43 GB), kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2v
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "stage_text or cli" > $O/tests_text.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 4
