#!/bin/bash
# round 3, call g4n: pass R with the readlanes interleaved into the SALU chain (filling its dependency gaps)
# the GPU suite, then the bench A/B against the readlanes-first build
# (fastqueeze_amd/lib/libseqarc_amd_rv11.so through SA_LIB), alternating, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4n
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
for i in 1 2; do
    timeout -k 10 300 $B > $O/il_$i.json 2> $O/il_$i.err || exit 2
    SA_LIB=$R/fastqueeze_amd/lib/libseqarc_amd_rv11.so timeout -k 10 300 $B > $O/rf_$i.json 2> $O/rf_$i.err || exit 3
done
