# Final per-session check on the GPU box: parity tests + smoke, then the
# default bench under rocprofv3 kernel stats and the two PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -3 gpurun_out/${TAG}_tests.log
bash scripts/gpu_r2.sh $TAG
