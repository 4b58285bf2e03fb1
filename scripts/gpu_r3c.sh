#!/bin/bash
# round 2, call r3c: device timeline of the end-to-end CLI run (rocprofv3 kernel trace of seqarc_amd -c on
# the bench's 43 GB PE pair) and one-context phase times (k_md5 with one batch in flight)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3c
mkdir -p $O
cd $R
export TMPDIR=/tmp
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u bench.py --contexts 1 --batches 1 --steps 4 --warmup 1 --e2e-batches 0 --cpu-seconds 0 > $O/b_c1.json 2> $O/b_c1.err || exit 1
timeout -k 10 600 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 2
SA_SYNC=block timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o cli -- fastqueeze_amd/bin/seqarc_amd -c -f -v -1 $D/r1.fq -2 $D/r2.fq -o $D/out --contexts 5 --batch 69 > $O/cli.out 2> $O/cli.err || exit 3
python3 scripts/e2e_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/timeline.txt || exit 4
