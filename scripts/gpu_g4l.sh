#!/bin/bash
# round 3, call g4l: the sort scatter with one tile buffer (keys, then values: 22 KB of LDS, three workgroups beside pass R instead of two)
# the GPU suite, then the bench A/B against the two-buffer build
# (fastqueeze_amd/lib/libseqarc_amd_s2.so through SA_LIB), alternating, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4l
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
for i in 1 2; do
    timeout -k 10 300 $B > $O/one_$i.json 2> $O/one_$i.err || exit 2
    SA_LIB=$R/fastqueeze_amd/lib/libseqarc_amd_s2.so timeout -k 10 300 $B > $O/two_$i.json 2> $O/two_$i.err || exit 3
done
