#!/bin/bash
# Round-4 small-n session (via gpurun from the repo root): the host-driver and
# thread-exit tests, bench.py --sweep, and the same sweep under a kernel trace
# (per-size kernel durations: tools/sweep_kernels.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_sweep
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
step pytest 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -k "host_driver or exited_threads" -x -v --timeout 120 --timeout-method thread
step sweep 300 python -u bench.py --sweep
cd /tmp && export TMPDIR=/tmp
step sweep_trace 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_sweep -o run --output-format csv -- python3 $R/bench.py --sweep
cp $(find /tmp/prof_sweep -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python3 $R/tools/sweep_kernels.py $(find /tmp/prof_sweep -name "*kernel_trace.csv" | head -1) > $OUT/sweep_kernels.txt
cat $OUT/sweep_kernels.txt
