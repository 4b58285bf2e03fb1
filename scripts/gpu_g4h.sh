#!/bin/bash
# round 3, call g4h: pass R's step with the record split per segment in the VALU (11 instructions a
# step instead of 12): the GPU suite, then the bench A/B against the 12-instruction build
# (fastqueeze_amd/lib/libseqarc_amd_r12.so through SA_LIB), alternating, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4h
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
for i in 1 2; do
    timeout -k 10 300 $B > $O/r11_$i.json 2> $O/r11_$i.err || exit 2
    SA_LIB=$R/fastqueeze_amd/lib/libseqarc_amd_r12.so timeout -k 10 300 $B > $O/r12_$i.json 2> $O/r12_$i.err || exit 3
done
