#!/bin/bash
# Round 6, third call: the deep-pass occupancy A/B over four CLV placements
# (tools/ab_deep_occ.hip) and the exact-protein tile-group A/B
# (tools/ab_prot_tiles.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 build/ab_deep_occ 20 3 > gpurun_out/r06_ab_deep_occ_place.log 2>&1 &&
timeout -k 10 200 build/ab_prot_tiles 262144 4099 1048576 > gpurun_out/r06_ab_prot_tiles.log 2>&1 &&
timeout -k 10 300 python3 -u tools/node_placement.py --sizes 16777216,50000000,100000000 --sets 3 --calls 7 > gpurun_out/r06_node_placement.log 2>&1
