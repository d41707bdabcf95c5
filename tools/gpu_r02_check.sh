#!/bin/bash
# Round-2 check session on the GPU box (run via gpurun from the repo root):
# the GPU test suite, then the default bench line (node, configs[1]) with its
# CPU baseline on the same inputs, then configs[3] at N = 1 (512 nodes x 2^20
# sites on one GPU, RCCL world 1 under torch.distributed.run).  Every GPU step
# has its own time limit; the script stops at the first step that faults,
# aborts or times out.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -2 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
cd $R
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_node 240 python -u bench.py --steps 200 --warmup 20
step nodes512 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29531 bench.py --workload nodes512 --steps 10 --warmup 2 --no-cpu-baseline
