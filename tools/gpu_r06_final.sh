#!/bin/bash
# Round 6 closing measurement session (via gpurun from the repo root):
#   1. the driver's exact command (default invocation: node line +
#      nodes512 / tree64 / protein / protein.exact sub-records), wall-timed;
#   2. the same command under rocprofv3 --kernel-trace --stats (the kernel
#      averages the line's fracs are checked against), summarised per launch
#      shape by tools/trace_by_grid.py (the host-array leg launches the node
#      kernel at other grids);
#   3. the N = 2 command shape at FULL size on the one GPU (gloo ranks
#      folded onto it; rates meaningless, checks and memory real);
# preceded by the whole GPU test suite on the same tree.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_final
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N) - $t0, 1))")" | tee -a $OUT/steps.txt
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name.log; exit $rc; fi
  return 0
}
cd $R
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
grep '^{' $OUT/bench_driver.log > $OUT/bench_driver.json
cd /tmp && export TMPDIR=/tmp
step bench_driver_rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5
cd $R
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/bench_driver_kernel_stats.csv \;
python3 tools/trace_by_grid.py $(find $OUT/prof -name "*kernel_trace.csv") $OUT/bench_driver_kernels_by_grid.json > /dev/null
gzip -c $(find $OUT/prof -name "*kernel_trace.csv") > $OUT/bench_driver_kernel_trace.csv.gz
rm -rf $OUT/prof
step rehearse_gloo2_full 900 env PLFX_DIST_BACKEND=gloo python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline
grep '^{' $OUT/rehearse_gloo2_full.log > $OUT/rehearse_gloo2_full.json
