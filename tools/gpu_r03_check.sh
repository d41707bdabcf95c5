#!/bin/bash
# Round-3 check (GPU box, via gpurun from the repo root): the GPU suite, smoke(),
# and the default bench lines of the node / nodes512 / protein workloads, each
# step under its own time limit; stops at the first failing step.
#   tools/gpu_r03_check.sh TAG [pytest selection...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -1 $OUT/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
cd $R
step pytest_gpu 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_node 300 python -u bench.py
step bench_nodes512 300 python -u bench.py --workload nodes512 --steps 10 --warmup 2 --no-cpu-baseline
step bench_protein 300 python -u bench.py --workload protein
