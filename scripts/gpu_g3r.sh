#!/bin/bash
# round 3, call g3r: R-Block 16-byte walks (lossy parity + ONT-shape bench), fused name columns A/B
# (SA_PREP_SPLIT), the CLI's kernel trace (--release: the profiler's own exit handlers must run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3r
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "lossy or ont or rblock or long" --timeout 120 --timeout-method thread > $O/parity_lossy.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/fused.json 2> $O/fused.err || exit 2
SA_PREP_SPLIT=1 timeout -k 10 300 $B > $O/split.json 2> $O/split.err || exit 3
timeout -k 10 300 $B > $O/fused2.json 2> $O/fused2.err || exit 4
timeout -k 10 400 python -u bench.py --ont --lossy 1.15 --pairs 60000 --steps 12 --e2e-batches 0 --cpu-seconds 0 > $O/ont.json 2> $O/ont.err || exit 5
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 6
sleep 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --contexts 5 --batch 69 --release > $O/cli_prof.log 2>&1 || exit 7
