#!/bin/bash
# round 2, call r3k: where the end-to-end run's last second goes (context teardown): the CLI on the bench's
# 43 GB pair with and without SA_FAST_EXIT, wall clock around each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3k
mkdir -p $O
cd $R
export TMPDIR=/tmp
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 600 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 1
for V in 0 1; do
    S=$(date +%s.%N)
    SA_FAST_EXIT=$V timeout -k 10 300 fastqueeze_amd/bin/seqarc_amd -c -f -v -1 $D/r1.fq -2 $D/r2.fq -o $D/out --contexts 5 --batch 69 > $O/cli_$V.out 2> $O/cli_$V.err || exit 2
    E=$(date +%s.%N)
    echo "fast_exit=$V wall $(python3 -c "print(round($E - $S, 3))") s" >> $O/wall.txt
    rm -f $D/out.arc
done
