#!/bin/bash
# round 4, call r4o: the bench (and the GPU tests) load libseqarc_amd after
# torch, so they run on torch's bundled HIP / HSA runtime (ROCm 7.0, same
# sonames); seqarc_amd links /opt/rocm's (7.2).  The CLI on 42.8 GB with the
# pass-R probe on each runtime: is the clock drop the runtime's?
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4o2}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
TL0=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
# torch ships libamdhip64.so / libhsa-runtime64.so (sonames .so.7 / .so.1):
# a directory of links under the soname file names, then torch's own lib dir
TL=/tmp/sa_torch_rt
mkdir -p $TL
ln -sf $TL0/libamdhip64.so $TL/libamdhip64.so.7
ln -sf $TL0/libhsa-runtime64.so $TL/libhsa-runtime64.so.1
TL=$TL:$TL0
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $SMI 2>/dev/null' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
sampler() {
    while true; do
        echo "t $(date +%s.%N)" >> $1
        timeout 5 rocm-smi --showpower --showclocks --showtemp --csv >> $1 2>&1
        sleep 0.5
    done
}
cli() {   # name, env...
    local name=$1; shift
    sleep 8
    sampler $O/smi_$name.txt & SMI=$!
    (cd $E && env "$@" SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    rm -f $E/e2e.arc
    echo "cli_$name rc=$rc" >> $O/steps.txt
    [ $rc -eq 0 ]
}
echo "torch lib: $TL" > $O/env.txt
ldd $R/fastqueeze_amd/bin/seqarc_amd >> $O/env.txt 2>&1
LD_LIBRARY_PATH=$TL ldd $R/fastqueeze_amd/bin/seqarc_amd >> $O/env.txt 2>&1
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
rm -rf $IN
cli rocm72 && cli torch70 LD_LIBRARY_PATH=$TL && cli rocm72b && cli torch70b LD_LIBRARY_PATH=$TL
python3 scripts/rv_probe.py $O/probe_rocm72.txt $O/probe_torch70.txt $O/probe_rocm72b.txt $O/probe_torch70b.txt > $O/probe_report.txt 2>&1
