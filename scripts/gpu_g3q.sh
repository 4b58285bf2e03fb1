#!/bin/bash
# round 3, call g3q: parity with the fused name columns (k_prep_sq16); the bench without e2e; the CLI on 42.8 GB
# with 4 vs 24 hardware queues, and its rocprofv3 kernel trace (parse kernels, pass R under the CLI's load)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3q
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" > $O/env.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify > $O/bench.json 2> $O/bench.err || exit 2
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 3
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --contexts 5 --batch 69"
sleep 3
GPU_MAX_HW_QUEUES=24 timeout -k 10 120 $CLI > $O/cli_q24.log 2>&1 || exit 4
sleep 8
GPU_MAX_HW_QUEUES=4 timeout -k 10 120 $CLI > $O/cli_q4.log 2>&1 || exit 5
sleep 8
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --contexts 5 --batch 69 > $O/cli_prof.log 2>&1 || exit 6
