#!/bin/bash
# round 3, call g3x: pass R with shared waves for the short chains: parity, bench A/B, CLI A/B on 42.8 GB (SA_RV_SHORT_WAVES=0:
# a wave per chain)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3x
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py tests/test_gpu_hash.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
B="python -u bench.py --steps 16 --e2e-batches 0 --cpu-seconds 0 --no-verify"
timeout -k 10 300 $B > $O/sh.json 2> $O/sh.err || exit 2
SA_RV_SHORT_WAVES=0 timeout -k 10 300 $B > $O/one.json 2> $O/one.err || exit 3
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
run cli_sh timeout -k 10 120 $CLI || exit 5
run cli_one SA_RV_SHORT_WAVES=0 timeout -k 10 120 $CLI || exit 6
run cli_sh2 timeout -k 10 120 $CLI || exit 7
