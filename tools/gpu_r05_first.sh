#!/bin/bash
# Round-5 first GPU pass (via gpurun from the repo root): the whole GPU suite
# (the new nodes512 sub-record and N>1 honesty fields are asserted in
# tests/test_gpu_dist.py), then the driver's own bench command with its wall
# time, then the same command under a rocprofv3 kernel trace.  Every step under
# its own time limit; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_first
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N) - $t0, 1))")"
  tail -1 $OUT/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then tail -30 $OUT/$name.log; exit $rc; fi
  return 0
}
cd $R
step pytest_gpu ${PYTEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS:-}
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step trace 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_r05 -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
cp $(find /tmp/prof_r05 -name "*kernel_stats.csv" | head -1) $OUT/bench_driver_kernel_stats.csv
head -8 $OUT/bench_driver_kernel_stats.csv
