#!/bin/bash
# Round-2 tuning session (GPU box, via gpurun from the repo root): the f32
# node-kernel grid/trip variants at 2^20 and 2^21 sites (tools/tune_f32.hip,
# built in-tree beforehand), and the box's CPU share for the CPU baseline.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02_tune}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -14 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
cd $R
{ cat /sys/fs/cgroup/cpu.max 2>&1; nproc; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}"; } > $OUT/cpu_share.log
cat $OUT/cpu_share.log
step tune_f32_20 180 ./build/tune_f32 1048576 60
step tune_f32_21 180 ./build/tune_f32 2097152 40
