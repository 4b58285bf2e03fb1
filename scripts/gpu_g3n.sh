#!/bin/bash
# round 3, call g3n: e2e legs (short ~18 GB, long 42.8 GB) with the reserve-slack fix, ramp vs --no-ramp;
# rocprofv3 kernel stats of the in-HBM bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3n
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
B="python -u bench.py --steps 16 --cpu-seconds 0 --no-verify --e2e-gz-blocks 0"
timeout -k 10 600 $B --e2e-log $O/e2e_ramp.log > $O/ramp.json 2> $O/ramp.err || exit 1
timeout -k 10 600 $B --e2e-log $O/e2e_noramp.log --e2e-args=--no-ramp > $O/noramp.json 2> $O/noramp.err || exit 2
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u $R/bench.py --steps 8 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/prof_bench.json 2> $O/prof_bench.err || exit 3
