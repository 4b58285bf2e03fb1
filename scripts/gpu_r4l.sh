#!/bin/bash
# round 4, call r4l: what lowers the shader clock under seqarc_amd -c (r4k:
# pinning during the run is not it; the bench's staged-text leg -- the same
# device work, driven from Python -- keeps 2.4 GHz).  (1) the CLI as is; (2) the
# CLI while a second process holds a torch context on the GPU and sleeps; (3)
# the bench's staged-text leg while the CLI's reader runs beside it in a loop
# (seqarc_amd --ingest-only: pread + cut, no device work).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r4l}
O=$R/gpurun_out/$TAG
IN=/dev/shm/sa_bench_inputs
E=/dev/shm/sa_cli_e2e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $IN $E; kill $SMI $BG 2>/dev/null' EXIT
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
cli() {   # name
    local name=$1; shift
    sampler $O/smi_$name.txt & SMI=$!
    (cd $E && SA_RV_PROBE=$O/probe_$name.txt timeout -k 10 120 $R/fastqueeze_amd/bin/seqarc_amd -c -f -v -t 16 \
        -1 r1.fq -2 r2.fq -o e2e --contexts 5 --batch 69 --slevel 3 --qlevel 2 --block-size 50) > $O/cli_$name.log 2>&1
    local rc=$?
    kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
    rm -f $E/e2e.arc
    echo "cli_$name rc=$rc" >> $O/steps.txt
    [ $rc -eq 0 ]
}
step write_inputs timeout -k 10 300 python -u bench.py --write-inputs $IN > $O/write_inputs.log 2>&1
mkdir -p $E
for k in 1 2 3; do for g in 0 1 2 3; do cat $IN/b${g}_r1.fq >> $E/r1.fq; cat $IN/b${g}_r2.fq >> $E/r2.fq; done; done
sleep 8
cli base || exit 3
sleep 8
timeout -k 5 90 python -u -c "import torch, time; torch.zeros(1, device='cuda'); print('torch holds the GPU', flush=True); time.sleep(80)" > $O/torch_holder.log 2>&1 & BG=$!
sleep 20
cli torch_beside
kill $BG 2>/dev/null; wait $BG 2>/dev/null
sleep 8
(for i in 1 2 3 4 5 6 7 8 9 10; do (cd $E && timeout -k 5 60 $R/fastqueeze_amd/bin/seqarc_amd -c -f -t 16 -1 r1.fq -2 r2.fq -o ing --contexts 5 --batch 69 --block-size 50 --devices 8 --ingest-only) >> $O/ingest_loop.log 2>&1; rm -f $E/ing.arc; done) & BG=$!
sleep 3
sampler $O/smi_staged_reader.txt & SMI=$!
SA_RV_PROBE=$O/probe_staged_reader.txt step staged_reader timeout -k 10 300 python -u bench.py --inputs $IN --no-legs --no-verify --steps 2 --warmup 0 --text-steps 30 > $O/staged_reader.json 2> $O/staged_reader.err
kill $SMI $BG 2>/dev/null; wait $SMI $BG 2>/dev/null
python3 scripts/rv_probe.py $O/probe_base.txt $O/probe_torch_beside.txt $O/probe_staged_reader.txt > $O/probe_report.txt 2>&1
