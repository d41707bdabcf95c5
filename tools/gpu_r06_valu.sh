#!/bin/bash
# Round 6: configs[4] on the VALU in FMA mode (PLFX_FMA | PLFX_VALU,
# plf_prot_valu.hip) -- its parity tests, then the protein bench lines
# alternated on one box: matrix cores, VALU FMA, exact.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-r06_valu}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_protein.py -x -q --timeout 240 --timeout-method thread -k "valu" > gpurun_out/$T/pytest.log 2>&1 &&
for r in 1 2; do
  for m in "" "--valu" "--exact"; do
    timeout -k 10 200 python3 -u bench.py --workload protein $m --no-cpu-baseline > gpurun_out/$T/bench_${r}${m}.json 2> gpurun_out/$T/bench_${r}${m}.err || exit 1
  done
done
