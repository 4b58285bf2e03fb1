#!/bin/bash
# round 2, call y: MD5 non-pipelined default; sweep of the pass-R LDS reservation and the wave-per-read grid
# on one box; default bench with the end-to-end leg and the CLI's per-batch device phases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2y
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "golden or reference or stage_text" > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 16"
timeout -k 10 600 $B > $O/b_def.json 2> $O/b_def.err || exit 2
SA_CODER_LDS=57344 timeout -k 10 600 $B > $O/b_lds56.json 2> $O/b_lds56.err || exit 3
SA_CODER_LDS=40960 timeout -k 10 600 $B > $O/b_lds40.json 2> $O/b_lds40.err || exit 4
SA_WAVE_GRID=16 timeout -k 10 600 $B > $O/b_grid16.json 2> $O/b_grid16.err || exit 5
timeout -k 10 900 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err || exit 6
