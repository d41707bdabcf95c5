#!/bin/bash
# Round 6: the exact VALU protein kernel without the register-held next tile
# -- the protein GPU tests, then its stamped PMC traffic record (tools/measure.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_exact_nopf
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_protein.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06_exact_nopf/pytest_protein.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06b_protein_exact 20 --workload protein --exact > gpurun_out/r06_exact_nopf/measure.log 2>&1
rc=$?
tail -2 gpurun_out/r06_exact_nopf/pytest_protein.log
grep -v "^$" gpurun_out/r06_exact_nopf/measure.log | cut -c1-220
exit $rc
