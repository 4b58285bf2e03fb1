#!/bin/bash
# round 2, call n: measurement set of the default bench -- kernel trace + stats, PMC traffic (FETCH_SIZE,
# WRITE_SIZE passes), Slevel 8 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2n
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --cpu-seconds 0 --e2e-batches 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run -- python3 -u bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-verify --e2e-batches 0 > $O/pmc_$C.json 2> $O/pmc_$C.err || exit 2
done
python3 scripts/pmc_traffic.py $(ls $O/pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/pmc_WRITE_SIZE/*counter_collection.csv | head -1) $O/traffic.json > $O/traffic.txt || exit 3
timeout -k 10 600 python -u bench.py --slevel 8 --cpu-seconds 0 --e2e-batches 0 > $O/slevel8.json 2> $O/slevel8.err || exit 4
