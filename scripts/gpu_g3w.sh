#!/bin/bash
# round 3, call g3w: mailbox copies as kernels (not SDMA): parity, bench A/B, CLI A/B on 42.8 GB (SA_MAIL_DMA=1:
# hipMemcpyAsync)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3w
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py tests/test_gpu_hash.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/kern.json 2> $O/kern.err || exit 2
SA_MAIL_DMA=1 timeout -k 10 300 $B > $O/dma.json 2> $O/dma.err || exit 3
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
run cli_kern timeout -k 10 120 $CLI || exit 5
run cli_dma SA_MAIL_DMA=1 timeout -k 10 120 $CLI || exit 6
run cli_kern2 timeout -k 10 120 $CLI || exit 7
