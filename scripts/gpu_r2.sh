# Round-2 measurement on the GPU box: rocprofv3 kernel stats of the default
# bench, then two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs per the
# MI355X_MICROARCH.md HBM recipe) -> per-launch traffic JSON.
# usage: bash scripts/gpu_r2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
    python3 -u $R/bench.py > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o run -- \
        python3 -u $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-verify \
        > $R/gpurun_out/pmc_${TAG}_$C.json 2> $R/gpurun_out/pmc_${TAG}_$C.err || exit 1
done
python3 $R/scripts/pmc_traffic.py $(ls $R/gpurun_out/pmc_${TAG}_FETCH_SIZE/*counter_collection.csv | head -1) \
    $(ls $R/gpurun_out/pmc_${TAG}_WRITE_SIZE/*counter_collection.csv | head -1) $R/gpurun_out/traffic_$TAG.json
cat $R/gpurun_out/${TAG}_bench.json
