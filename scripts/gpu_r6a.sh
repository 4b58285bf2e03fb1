#!/bin/bash
# round 6, call r6a: feed_probe -- cycles per symbol of pass R's range chain
# under seven ways of feeding the scalar unit (scripts/micro/feed_probe.hip)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r6a}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 240 ./scripts/micro/feed_probe 1048576 > $O/feed_probe.txt 2>&1
