# rocprofv3 kernel-trace summary of the default bench (run on the GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- \
    python3 -u $R/bench.py --steps 2 --warmup 1 --cpu-seconds 10 ${BENCH_ARGS} \
    > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err
