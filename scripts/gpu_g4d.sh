#!/bin/bash
# round 3, call g4d: stage-ahead CLI (each context stages its next batch while encoding): GPU CLI tests, then the
# CLI on 42.8 GB: 5 contexts without stage-ahead, 4 and 5 with
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4d
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_align.py -x -q -k "cli or stage" --timeout 120 --timeout-method thread > $O/parity_cli.log 2>&1 || exit 1
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 2
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --batch 69"
run() {
    local n=$1; shift
    sleep 8
    local t0=$(date +%s.%N)
    env "$@" > $O/$n.log 2>&1 || return 1
    local t1=$(date +%s.%N)
    echo "$n wall $(python3 -c "print(round($t1 - $t0, 3))") s" >> $O/walls.txt
}
run c5_nosa timeout -k 10 120 $CLI --contexts 5 --no-stage-ahead || exit 3
run c4_sa timeout -k 10 120 $CLI --contexts 4 || exit 4
run c5_sa timeout -k 10 120 $CLI --contexts 5 || exit 5
run c5_nosa2 timeout -k 10 120 $CLI --contexts 5 --no-stage-ahead || exit 6
run c4_sa2 timeout -k 10 120 $CLI --contexts 4 || exit 7
md5sum $D/e2e.arc > $O/arc_md5.txt 2>&1 || true
