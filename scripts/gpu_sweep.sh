# Bench sweep over tuning environment settings (one bench run each).
# usage: bash scripts/gpu_sweep.sh TAG "ENV1=a ENV2=b" "ENV1=c" ... -- bench args
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cfgs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p $R/gpurun_out
cd $R
for c in "${cfgs[@]}"; do
    echo "== $c" | tee -a gpurun_out/${TAG}_sweep.txt
    env $c timeout -k 10 300 python3 -u bench.py "$@" 2>>gpurun_out/${TAG}_sweep.err | tee -a gpurun_out/${TAG}_sweep.txt || exit 1
done
