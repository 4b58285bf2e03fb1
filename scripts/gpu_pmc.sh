# PMC pass over a short bench run (one counter group per rocprofv3 run).
# usage: bash scripts/gpu_pmc.sh TAG "COUNTERS" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
CTRS=$1; shift
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- \
    python3 -u $R/bench.py "$@" > $R/gpurun_out/pmc_${TAG}_bench.json 2> $R/gpurun_out/pmc_${TAG}_bench.err
