#!/bin/bash
# round 5, call r5a: the host ingest building blocks (scripts/ingest_probe.cpp:
# pread into pinned memory, mmap fault-in, hipHostRegister of a mapped file,
# DMA from it, newline counting, a zero-copy kernel) and amd-smi's metric
# fields (help + one snapshot) for the throttle record.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5a}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
trap 'rm -f /dev/shm/ingest_probe.fq' EXIT
(timeout 60 amd-smi metric --help; timeout 60 amd-smi monitor --help) > $O/amdsmi_help.txt 2>&1
timeout 60 amd-smi metric -g 0 > $O/amdsmi_metric.txt 2>&1
timeout 60 amd-smi metric -g 0 --json > $O/amdsmi_metric.json 2>&1
nproc > $O/host.txt; cat /sys/fs/cgroup/cpu.max >> $O/host.txt 2>&1; free -g >> $O/host.txt; cat /sys/kernel/mm/transparent_hugepage/shmem_enabled >> $O/host.txt 2>&1; uname -a >> $O/host.txt
timeout -k 10 400 scripts/bin/ingest_probe /dev/shm/ingest_probe.fq 12 > $O/ingest_probe.txt 2>&1
echo "probe rc=$?" >> $O/steps.txt
