#!/bin/bash
# round 3, call g3e: the hash tests alone (teardown hang hunt), then the GPU parity suite with k_emit_sq16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3e
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
timeout -k 10 170 python -u -X faulthandler -m pytest tests/test_gpu_hash.py -x -v --timeout 100 --timeout-method thread > $O/hash.log 2>&1
echo "hash rc=$?" >> $O/hash.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread > $O/parity.log 2>&1 || exit 2
