#!/bin/bash
# round 3, call g4b: host-side waits between a context's streams (SA_HOST_WAITS=0: barrier packets): parity, bench
# A/B with hardware queues 4 (the boxes' preset) / 8 / 24, CLI A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4b
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py tests/test_gpu_hash.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
i=0
for v in "SA_HOST_WAITS=1 GPU_MAX_HW_QUEUES=4" "SA_HOST_WAITS=0 GPU_MAX_HW_QUEUES=4" "SA_HOST_WAITS=1 GPU_MAX_HW_QUEUES=8" \
         "SA_HOST_WAITS=1 GPU_MAX_HW_QUEUES=24" "SA_HOST_WAITS=1 GPU_MAX_HW_QUEUES=4" "SA_HOST_WAITS=0 GPU_MAX_HW_QUEUES=4"; do
    i=$((i + 1))
    echo "$i $v" >> $O/variants.txt
    env $v timeout -k 10 300 $B > $O/b$i.json 2> $O/b$i.err || exit 2
done
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 4
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --batch 69 --contexts 5"
run() {
    local n=$1; shift
    sleep 8
    local t0=$(date +%s.%N)
    env "$@" > $O/$n.log 2>&1 || return 1
    local t1=$(date +%s.%N)
    echo "$n wall $(python3 -c "print(round($t1 - $t0, 3))") s" >> $O/walls.txt
}
run cli_hw timeout -k 10 120 $CLI || exit 5
run cli_dev SA_HOST_WAITS=0 timeout -k 10 120 $CLI || exit 6
run cli_hw2 timeout -k 10 120 $CLI || exit 7
run cli_dev2 SA_HOST_WAITS=0 timeout -k 10 120 $CLI || exit 8
