#!/bin/bash
# round 2, call l: contexts 6, MD5 priority off, kernel-trace CSV of the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2l
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python -u bench.py --cpu-seconds 0 --no-verify --e2e-batches 0"
timeout -k 10 600 $B --contexts 5 > $O/c5.json 2> $O/c5.err || exit 1
SA_MD5_PRIO=0 timeout -k 10 600 $B --contexts 5 > $O/c5_md5p0.json 2> $O/c5_md5p0.err || exit 2
timeout -k 10 600 $B --contexts 6 > $O/c6.json 2> $O/c6.err || exit 3
SA_MD5_PRIO=0 timeout -k 10 600 $B --contexts 6 > $O/c6_md5p0.json 2> $O/c6_md5p0.err || exit 4
