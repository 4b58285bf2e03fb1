#!/bin/bash
# round 2, call r3p: SEQ keys carry the base (values implicit in the first sort pass) for k <= 14 -- GPU suite,
# then A/B against SA_SEQ_PACK=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3p
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
B="python -u bench.py --e2e-batches 0 --cpu-seconds 0 --steps 24"
timeout -k 10 600 $B > $O/b_pack.json 2> $O/b_pack.err || exit 3
SA_SEQ_PACK=0 timeout -k 10 600 $B > $O/b_nopack.json 2> $O/b_nopack.err || exit 4
timeout -k 10 600 $B > $O/b_pack2.json 2> $O/b_pack2.err || exit 5
