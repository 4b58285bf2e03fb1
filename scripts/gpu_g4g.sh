#!/bin/bash
# round 3, call g4g: pass R alone on a 69-block batch, in the bench (one context) and in the command
# line (one context, no ramp); the command line with host parsing; then the bench's end-to-end legs
# with compress() exiting before its destructors (the 1.35 s between the CLI's clock and its exit, g4f).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4g
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 400 python -u bench.py --contexts 1 --steps 4 --warmup 1 --e2e-batches 0 --cpu-seconds 0 --no-verify \
    > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 2
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --slevel 3 --qlevel 2"
sleep 8
timeout -k 10 200 $CLI --contexts 1 --batch 69 --no-ramp > $O/cli_c1.log 2>&1 || exit 3
sleep 8
timeout -k 10 200 $CLI --contexts 5 --batch 69 --host-parse > $O/cli_hostparse.log 2>&1 || exit 4
rm -rf $D
timeout -k 10 900 python -u bench.py --steps 8 --cpu-seconds 0 --no-verify --e2e-log $O/e2e.log \
    > $O/bench_e2e.json 2> $O/bench_e2e.err || exit 5
