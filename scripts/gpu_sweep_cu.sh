# Sensitivity of the default bench to the long-run CU split (SA_LONG_CU_EVERY).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for E in 3 5 8; do
    SA_LONG_CU_EVERY=$E timeout -k 10 300 python3 -u $R/bench.py --cpu-seconds 0 --no-verify --steps 2 \
        > $R/gpurun_out/cu_$E.json 2> $R/gpurun_out/cu_$E.err || exit 1
    python3 -c "import json;d=json.load(open('$R/gpurun_out/cu_$E.json'));print($E, d['value'], d['ms_per_step'], d['phase_ms']['coder_r'], d['phase_ms']['replay_aux'])"
done
