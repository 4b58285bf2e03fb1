# Round-3 check: parity tests + smoke, then the default (SE) bench and the
# --paired (150 bp PE) bench.  usage: bash scripts/gpu_r3.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py --paired --cpu-seconds 0 > gpurun_out/${TAG}_bench_pe.json 2> gpurun_out/${TAG}_bench_pe.err || exit 1
cat gpurun_out/${TAG}_bench_pe.json
