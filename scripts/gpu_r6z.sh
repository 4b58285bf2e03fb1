#!/bin/bash
# round 6, call r6z: where the command line's exit time goes (bench.py's
# exit_to_reaped_s, ~0.34 s of the 17.8 GB leg): the default against the exit
# probe (the output pool's buffers freed and the contexts released before the
# exit, each timed) and against no output pool (SA_CLI_OUT_POOL=0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
rm -rf $IN
step ab timeout -k 10 600 python3 -u scripts/cli_exit_ab.py $E/s $O/exit_ab.txt \
    def1= probe1=SA_CLI_EXIT_PROBE:1 def2= probe2=SA_CLI_EXIT_PROBE:1 nopool=SA_CLI_OUT_POOL:0 \
    def3= probe3=SA_CLI_EXIT_PROBE:1
