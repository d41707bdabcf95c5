#!/bin/bash
# Round 6: configs[4] exact mode with the matrices as scalar operands
# (PLFX_EXACT | PLFX_VALU, plf_prot_valu_exact.hip): parity, then its forms
# (PLFX_EXACT_FORM) against the LDS-matrix exact kernel, alternated, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r06_exact_forms}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_protein.py -x -q --timeout 240 --timeout-method thread -k "valu" > gpurun_out/$T/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python3 -u bench.py --workload protein --exact --no-cpu-baseline > gpurun_out/$T/lds_$r.json 2> gpurun_out/$T/lds_$r.err || exit 1
  for f in 1 2 3 4 5; do
    PLFX_EXACT_FORM=$f timeout -k 10 120 python3 -u bench.py --workload protein --exact --valu --no-cpu-baseline > gpurun_out/$T/form${f}_$r.json 2> gpurun_out/$T/form${f}_$r.err || exit 1
  done
done
