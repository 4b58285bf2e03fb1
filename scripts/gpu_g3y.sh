#!/bin/bash
# round 3, call g3y: does a 3.6 GB H2D copy slow the kernels beside it (dma_probe)?  Is the CLI process
# throttled by the cgroup CPU quota (cpu.stat around a run)?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3y
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 120 ./micro_run/dma_probe > $O/dma_probe.txt 2>&1 || exit 1
D=/dev/shm/sa_e2e_$$
trap 'rm -rf $D' EXIT
timeout -k 10 300 python -u scripts/make_e2e_files.py $D 4 3 > $O/make.log 2>&1 || exit 2
CLI="./fastqueeze_amd/bin/seqarc_amd -c -f -v -1 $D/r1.fq -2 $D/r2.fq -o $D/e2e --batch 69 --contexts 5"
sleep 8
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_before.txt 2>&1; cat /sys/fs/cgroup/cpu.max >> $O/cpu_stat_before.txt 2>&1
timeout -k 10 120 $CLI -t 16 > $O/cli_t16.log 2>&1 || exit 3
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_after.txt 2>&1
sleep 8
timeout -k 10 120 $CLI -t 4 > $O/cli_t4.log 2>&1 || exit 4
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_after2.txt 2>&1
