#!/bin/bash
# Round 6, second call: the deep-pass occupancy A/B (tools/ab_deep_occ.hip),
# then the GPU tests touched this round (dist, segment cap, tree).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 build/ab_deep_occ 20 5 > gpurun_out/r06_ab_deep_occ.log 2>&1 &&
timeout -k 10 120 build/ab_deep_occ 24 2 >> gpurun_out/r06_ab_deep_occ.log 2>&1 &&
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "dist or segment" > gpurun_out/r06_dist2.log 2>&1
