#!/bin/bash
# round 2, call r3a: AUX values implicit in the first sort pass (GPU suite), then the pipeline-depth sweep:
# more encoder contexts with smaller batches (the tail -- pass R, ~1 s -- is the same for any batch size)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0"
timeout -k 10 600 $B --steps 16 > $O/b_c5.json 2> $O/b_c5.err || exit 2
timeout -k 10 600 $B --steps 24 --contexts 8 --pairs 3100000 > $O/b_c8.json 2> $O/b_c8.err || exit 3
timeout -k 10 600 $B --steps 32 --contexts 10 --pairs 2500000 > $O/b_c10.json 2> $O/b_c10.err || exit 4
timeout -k 10 600 $B --steps 40 --contexts 12 --pairs 2000000 > $O/b_c12.json 2> $O/b_c12.err || exit 5
