#!/bin/bash
# One measurement session on the GPU box (run via gpurun from the repo root):
# parity tests, bench.py, rocprofv3 kernel trace + stats of the same bench
# command, and two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit in one
# pass on gfx950).  Every GPU step has its own time limit; the script stops at
# the first step that faults, aborts or times out.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out
mkdir -p $OUT
BENCH="$R/bench.py --steps 200 --warmup 20"
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if [ $rc -eq 1 ] && [ "$name" != "pytest_gpu" ]; then exit 1; fi
  return 0
}
cd $R
step pytest_gpu 900 python -m pytest tests -m gpu -q
tail -3 $OUT/pytest_gpu.log
step bench 300 python $BENCH
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
step prof_trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_trace -o run --output-format csv -- python3 $BENCH --no-cpu-baseline
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/prof_fetch -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 4 --no-cpu-baseline --launch bound
step prof_write 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/prof_write -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 4 --no-cpu-baseline --launch bound
find $OUT/prof_trace $OUT/prof_fetch $OUT/prof_write -name "*.csv" | head -20
python3 $R/tools/pmc_traffic.py $OUT/prof_fetch/run_counter_collection.csv $OUT/prof_write/run_counter_collection.csv $OUT/pmc_traffic.json > /dev/null && echo traffic ok
