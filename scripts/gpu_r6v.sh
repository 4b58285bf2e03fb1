#!/bin/bash
# round 6, call r6v: why the bench's ONT leg has ~60 ms of prep+scan where two
# ONT batches through the headline's pipeline have ~44: the leg (after a
# 2-step headline) and the ONT headline, each under the kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6v}
O=$R/gpurun_out/$TAG
INO=/dev/shm/sa_ont_inputs
mkdir -p $O
cd $R
export TMPDIR=/tmp SA_NO_BUILD=1
trap 'rm -rf $INO' EXIT
step() {
    local name=$1; shift
    local t0=$SECONDS
    "$@"; local rc=$?
    echo "$name rc=$rc $((SECONDS - t0))s" >> $O/steps.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
}
cd /tmp
step leg timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/leg -o run -- python3 -u $R/bench.py --steps 2 --warmup 1 --text-leg 0 --se-leg 0 --hash-leg 0 --e2e-batches 0 --ingest-devices 0 --cpu-seconds 0 > $O/leg.json 2> $O/leg.err
cd $R
step write_ont timeout -k 10 300 python -u bench.py --write-inputs $INO --ont --lossy 1.15 --batches 2 > $O/write_ont.log 2>&1
cd /tmp
step head timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o run -- python3 -u $R/bench.py --inputs $INO --ont --lossy 1.15 --batches 2 --no-legs --steps 10 > $O/head.json 2> $O/head.err
cd $R
python3 - $O > $O/compare.txt 2>&1 <<'PY'
import csv, glob, statistics, sys, collections
O = sys.argv[1]
for name in ("leg", "head"):
    f = glob.glob(f"{O}/{name}/*kernel_trace.csv")[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sa::", "")
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print("==", name)
    for n in sorted(d):
        if any(x in n for x in ("rb_", "prep", "scan_reads", "emit", "coder_rv", "md5", "aux_long")):
            v = d[n]
            print("%-40s n %4d med %8.2f mean %8.2f min %8.2f" % (n[:40], len(v), statistics.median(v), statistics.mean(v), min(v)))
PY
find $O -name '*kernel_trace.csv' -delete
find $O -name '*.csv' -size +4M -delete
true
