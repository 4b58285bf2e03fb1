#!/bin/bash
# round 3: g3t then g3u in one call (the pool is congested)
bash scripts/gpu_g3t.sh || exit $?
bash scripts/gpu_g3u.sh || exit $((10 + $?))
