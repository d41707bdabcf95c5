#!/bin/bash
# Round 6: the protein kernels as adopted (f64 exact on the scalar-operand
# kernel; FMA on the VALU) -- protein GPU tests, their stamped PMC traffic
# records (tools/measure.sh), then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_prot_records
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_protein.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06_prot_records/pytest_protein.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06_protein_exact 20 --workload protein --exact > gpurun_out/r06_prot_records/measure_exact.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06_protein_valu 20 --workload protein --valu > gpurun_out/r06_prot_records/measure_valu.log 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_prot_records/pytest_gpu.log 2>&1
