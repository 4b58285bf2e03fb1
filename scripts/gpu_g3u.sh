#!/bin/bash
# round 3, call g3u: the CLI on 42.8 GB: host wait mode (SA_SYNC block vs spin), pass R partitioned per
# context (SA_RV_PART=1), 4 vs 5 contexts; device settled 8 s before each run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3u
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 1
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --batch 69"
run() {   # name, env..., then CLI args after --
    local n=$1; shift
    sleep 8
    local t0=$(date +%s.%N)
    env "$@" > $O/$n.log 2>&1 || return 1
    local t1=$(date +%s.%N)
    echo "$n wall $(python3 -c "print(round($t1 - $t0, 3))") s" >> $O/walls.txt
}
run block timeout -k 10 120 $CLI --contexts 5 || exit 2
run spin SA_SYNC=spin timeout -k 10 120 $CLI --contexts 5 || exit 3
run part SA_RV_PART=1 timeout -k 10 120 $CLI --contexts 5 || exit 4
run c4 timeout -k 10 120 $CLI --contexts 4 || exit 5
run block2 timeout -k 10 120 $CLI --contexts 5 || exit 6
