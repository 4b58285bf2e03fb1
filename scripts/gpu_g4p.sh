#!/bin/bash
# round 3, call g4p: rocprofv3 kernel statistics of the committed tree (default bench, no e2e / cpu legs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4p
mkdir -p $O
cd /tmp
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u $R/bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/prof_bench.json 2> $O/prof_bench.err || exit 5
python3 $R/scripts/kstats_csv.py $O/prof > $O/kernel_stats.txt 2>&1 || true
