#!/bin/bash
# Round 6: the whole GPU suite + smoke() on the current tree, then the node
# placement / mapping table on this box with the current thresholds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_suite.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u tools/node_placement.py --sizes 33554432,50000000,100000000 --sets 3 --calls 7 > gpurun_out/r06_node_placement2.log 2>&1
