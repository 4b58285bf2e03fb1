#!/bin/bash
# round 2, call r3t: final tree -- smoke, default bench line (with e2e), kernel stats of the ONT lossy line after the R-Block carry guess
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3t
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/b.json 2> $O/b.err || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ont -- python3 -u bench.py --ont --lossy 1.15 --e2e-batches 0 --cpu-seconds 0 --steps 6 > $O/b_ont.json 2> $O/b_ont.err || exit 3
