#!/bin/bash
# round 5, call r5c: the GPU suite (segment reader, SWAR N-gap pass, AUX records
# zeroed in the tail), the default bench with every leg (SE leg new), then the
# kernel statistics of one context alone (no pipeline overlap: the front
# kernels' own times).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5c}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap "rm -rf $IN /dev/shm/sa_cli_e2e" EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc > $O/tests.log 2>&1
step bench timeout -k 10 720 python -u bench.py --e2e-log $O/e2e.log > $O/bench.json 2> $O/bench.err
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
step solo_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/solo_prof -o solo -- python3 -u bench.py --inputs $IN --no-legs --no-verify --contexts 1 --steps 4 --warmup 1 > $O/solo.json 2> $O/solo.err
# the CLI on the 42.8 GB files under a kernel + memory-copy trace (where the
# front kernels wait: DMA barriers, queue order), and the staged-text leg alone
E=/dev/shm/sa_cli_e2e
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
step text_trace timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/text_prof -o text -- python3 -u bench.py --inputs $IN --no-verify --steps 4 --warmup 1 --e2e-batches 0 --ont-leg 0 --hash-leg 0 --se-leg 0 --ingest-devices 0 --cpu-seconds 0 --decode-check 0 > $O/text.json 2> $O/text.err
rm -rf $IN
sleep 5
step cli_trace timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/cli_prof -o cli -- $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 -1 $E/r1.fq -2 $E/r2.fq -o $E/e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50 > $O/cli_trace.log 2>&1
rm -rf $E
