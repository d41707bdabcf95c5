#!/bin/bash
# Round 6: the VALU FMA protein kernel's forms (PLFX_VALU_FORM, plf_prot_valu.hip)
# alternated on one box, bench --workload protein --valu (2000 steps), twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r06_valu_forms}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2; do
  for f in ${FORMS:-0 1 2 3 4 5 6 7 8}; do
    PLFX_VALU_FORM=$f timeout -k 10 120 python3 -u bench.py --workload protein --valu --no-cpu-baseline > gpurun_out/$T/form${f}_$r.json 2> gpurun_out/$T/form${f}_$r.err || exit 1
  done
done
