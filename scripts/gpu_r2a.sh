#!/bin/bash
# round 2, call a: GPU parity tests, then the bench without and with pipelining
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --contexts 1 --cpu-seconds 0 > $O/bench_c1.json 2> $O/bench_c1.err || exit 2
timeout -k 10 600 python -u bench.py --contexts 2 > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
