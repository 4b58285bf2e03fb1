# Sweep of the pass R prefetch distance (SA_PF_SEGS) on the default bench.
# usage: bash scripts/gpu_sweep_pf.sh TAG "2 4 8 16"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VALS=$2
mkdir -p $R/gpurun_out
cd $R
for v in $VALS; do
    SA_PF_SEGS=$v timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-verify --steps 3 \
        > gpurun_out/${TAG}_pf$v.json 2> gpurun_out/${TAG}_pf$v.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pf', sys.argv[2], d['value'], d['phase_ms']['coder_r'])" \
        gpurun_out/${TAG}_pf$v.json $v
done
