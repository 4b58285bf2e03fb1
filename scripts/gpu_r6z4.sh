#!/bin/bash
# round 6, call r6z4: the command line's output buffers sized by the encoded
# blocks (sa_fetch_sizes, default) against their output bounds
# (SA_CLI_OUT_EXACT=0): exit -> reaped and wall on 17.8 GB and 42.8 GB,
# interleaved, the archives' MD5s compared; the CLI GPU tests first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6z4}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1 AB_MD5=1
trap 'rm -rf $IN $E' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -o cache_dir=/tmp/pyc -k "cli" > $O/tests.log 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E/s $E/l
for g in 0 1 2 3 0; do cat $IN/b${g}_r1.fq >> $E/s/r1.fq; cat $IN/b${g}_r2.fq >> $E/s/r2.fq; done
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/l/r1.fq; cat $IN/b${g}_r2.fq >> $E/l/r2.fq; done; done
rm -rf $IN
B=SA_CLI_OUT_EXACT:0
step short timeout -k 10 600 python3 -u scripts/cli_exit_ab.py $E/s $O/short_ab.txt \
    exact1= bound1=$B exact2= bound2=$B exact3= bound3=$B
step long timeout -k 10 600 python3 -u scripts/cli_exit_ab.py $E/l $O/long_ab.txt \
    exact1= bound1=$B exact2= bound2=$B
