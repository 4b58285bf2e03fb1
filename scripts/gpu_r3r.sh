#!/bin/bash
# round 2, call r3r: kernel stats of the configs[4]-shape line (ONT-like long reads, -l 1.15)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3r
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ont -- python3 -u bench.py --ont --lossy 1.15 --e2e-batches 0 --cpu-seconds 0 --steps 6 > $O/b_ont.json 2> $O/b_ont.err || exit 1
