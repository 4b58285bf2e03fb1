#!/bin/bash
# round 4, call r4j: instruction mix and stall shares of the front kernels
# (SQ counters, one rocprofv3 --pmc pass each of at most 8 SQ counters), on
# inputs written first by a process that never touches the GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4j}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN' EXIT
timeout -k 10 300 python -u bench.py --write-inputs $IN --batches 2 > $O/write_inputs.log 2>&1 || exit 1
cd /tmp
B="$R/bench.py --inputs $IN --batches 2 --no-legs --no-verify --steps 2 --warmup 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_a -o run -- python3 -u $B > $O/pmc_a.json 2> $O/pmc_a.err || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/pmc_b -o run -- python3 -u $B > $O/pmc_b.json 2> $O/pmc_b.err || exit 3
