set -o pipefail
mkdir -p gpurun_out
rocminfo | grep -m3 gfx > gpurun_out/g1_info.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --reads 2000000 --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err
