#!/bin/bash
# round 2, call h: pass-R variants at 4 contexts; end-to-end over all 4 batches (14 GB in /dev/shm)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2h
mkdir -p $O
cd $R
B="timeout -k 10 900 python -u bench.py --contexts 4 --cpu-seconds 0 --no-verify --e2e-batches 0"
timeout -k 10 900 python -u bench.py --contexts 4 --cpu-seconds 0 > $O/c4_e2e.json 2> $O/c4_e2e.err || exit 1
SA_CODER_VGPR=0 SA_CODER_WAVES=1 SA_CODER_LDS=0 $B > $O/salu_w1_pf4.json 2> $O/salu_w1_pf4.err || exit 2
SA_CODER_VGPR=0 SA_CODER_WAVES=1 SA_CODER_LDS=0 SA_PF_SEGS=2 $B > $O/salu_w1_pf2.json 2> $O/salu_w1_pf2.err || exit 3
SA_CODER_VGPR=0 SA_CODER_WAVES=4 SA_PF_SEGS=2 $B > $O/salu_w4_pf2.json 2> $O/salu_w4_pf2.err || exit 4
SA_CODER_VGPR=0 SA_CODER_WAVES=2 SA_CODER_LDS=61440 $B > $O/salu_w2.json 2> $O/salu_w2.err || exit 5
SA_CODER_WAVES=2 SA_CODER_LDS=61440 $B > $O/vgpr_w2.json 2> $O/vgpr_w2.err || exit 6
