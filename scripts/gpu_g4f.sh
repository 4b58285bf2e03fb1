#!/bin/bash
# round 3, call g4f: why is pass R 1.2-1.4 s per batch in the command line against 0.8 s in the
# bench?  The 12-batch stream (42.8 GB) through seqarc_amd with one knob changed per run: host sync
# mode (spin instead of block), stream-side waits instead of host waits, 4 contexts, 35-block
# batches; each run's -v log has the per-batch device phase times and the process start / exit stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g4f
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 2
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -t 16 -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --slevel 3 --qlevel 2"
run() {   # name, env..., -- extra args
    local name=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done
    shift
    sleep 8
    local t0=$(date +%s.%N)
    env "${envs[@]}" timeout -k 10 120 $CLI "$@" > $O/$name.log 2>&1 || return 1
    local t1=$(date +%s.%N)
    echo "$name wall $(awk "BEGIN{print $t1 - $t0}") s: $(tail -1 $O/$name.log)" | tee -a $O/summary.txt
}
run base X=1 -- -v --contexts 5 --batch 69 || exit 3
run spin SA_SYNC=spin -- -v --contexts 5 --batch 69 || exit 4
run streamwaits SA_HOST_WAITS=0 -- -v --contexts 5 --batch 69 || exit 5
run c4 X=1 -- -v --contexts 4 --batch 69 || exit 6
run b35 X=1 -- -v --contexts 5 --batch 35 || exit 7
run quiet X=1 -- --contexts 5 --batch 69 || exit 8
run base2 X=1 -- -v --contexts 5 --batch 69 || exit 9
