# GPU check: parity tests, then the default bench under rocprofv3 kernel trace.
# usage: bash scripts/gpu_round.sh TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}; shift
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
    python3 -u $R/bench.py "$@" > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err
rc=$?
tail -3 $R/gpurun_out/${TAG}_bench.err
cat $R/gpurun_out/${TAG}_bench.json
exit $rc
