#!/bin/bash
# round 3, call g3d: step trace of the reference path on the GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g3d
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1 SA_ALN_TRACE=1
timeout -k 10 170 python -u scripts/dbg_align.py > $O/se.log 2>&1 || exit 1
timeout -k 10 170 python -u scripts/dbg_align.py pe > $O/pe.log 2>&1 || exit 2
