#!/bin/bash
# Round-5 second GPU pass (via gpurun from the repo root): the new tests first
# (RCCL in the C++ drivers, destroy after the caller's stream is gone, lazy
# tables), then the whole GPU suite, the f64 VALU plateau probe (VERDICT r04
# item 4), the per-call sweep (cost of the per-workspace event), and the C++
# tree driver at 64 taxa x 2^20 sites with its RCCL reduction.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_second
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N) - $t0, 1))")"
  tail -1 $OUT/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name.log; exit $rc; fi
  return 0
}
cd $R
step pytest_new 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_api.py -k "destroy or lazy_tables or exited_threads or rccl or driver_end" tests/test_gpu_tree.py tests/test_gpu_parity.py::test_host_driver_end_to_end
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step valu_probe 240 ./build/valu_f64
step sweep 300 python -u bench.py --sweep
B=amd-versal-phylogenetic-likelihood-function_amd/build
step tree_rccl 300 $B/plfx_tree 64 1048576 20 --devices 0 --reduce rccl
step tree_host 300 $B/plfx_tree 64 1048576 20 --devices 0 --reduce host
step host_rccl 300 $B/plfx_host 1048576 10 4 --reduce rccl
