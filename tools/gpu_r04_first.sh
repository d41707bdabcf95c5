#!/bin/bash
# Round-4 first GPU pass (via gpurun from the repo root): the new standalone
# `bench.py --gpus 2` test, the node bench line plus a stamped PMC traffic
# record of its kernel, and the protein exact bench line.  Every step under its
# own time limit; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_first
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -1 $OUT/$name.log | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
cd $R
step pytest_selfl 300 python -u -m pytest tests/test_gpu_dist.py -k "without_outer_launcher" -x -v --timeout 240 --timeout-method thread
KERNEL=plf_dna_f64_pair_kernel timeout -k 10 900 bash tools/gpu_r03_measure.sh r04_node 20 > $OUT/measure_node.log 2>&1 || { echo "measure_node failed"; tail -20 $OUT/measure_node.log; exit 1; }
tail -8 $OUT/measure_node.log
cd $R
step bench_protein_exact 300 python -u bench.py --workload protein --exact
