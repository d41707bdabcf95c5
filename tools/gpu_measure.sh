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
# tree64 (configs[2], one fused six-level pass): kernel trace and the two PMC passes
TREE="$R/bench.py --workload tree64 --no-cpu-baseline"
step tree_bench 300 python $TREE --steps 50 --warmup 5
tail -1 $OUT/tree_bench.log
step tree_trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/tree_trace -o run --output-format csv -- python3 $TREE --steps 50 --warmup 5
step tree_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/tree_fetch -o run --output-format csv -- python3 $TREE --steps 20 --warmup 2 --launch bound
step tree_write 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/tree_write -o run --output-format csv -- python3 $TREE --steps 20 --warmup 2 --launch bound
ALG=$(python3 -c "import json; d=json.loads(open('$OUT/tree_bench.log').read().strip().splitlines()[-1]); print(d['roofline']['bytes_per_step'])")
python3 $R/tools/pmc_step.py $OUT/tree_fetch/run_counter_collection.csv $OUT/tree_write/run_counter_collection.csv $OUT/tree_pmc_traffic.json --steps 22 --alg-bytes $ALG > /dev/null && echo tree traffic ok

# protein (configs[4], FMA on the f64 matrix cores) and nodes64 (configs[3]'s
# per-GPU shard): bench line, kernel trace, the two PMC passes, per-step traffic
for W in protein nodes64; do
  case $W in protein) K=100; P=20 ;; nodes64) K=20; P=6 ;; esac
  WB="$R/bench.py --workload $W --no-cpu-baseline"
  step ${W}_bench 300 python $WB --steps $K --warmup 5
  tail -1 $OUT/${W}_bench.log
  step ${W}_trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/${W}_trace -o run --output-format csv -- python3 $WB --steps $K --warmup 5
  step ${W}_fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/${W}_fetch -o run --output-format csv -- python3 $WB --steps $P --warmup 2 --launch bound
  step ${W}_write 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/${W}_write -o run --output-format csv -- python3 $WB --steps $P --warmup 2 --launch bound
  ALG=$(python3 -c "import json; d=json.loads(open('$OUT/${W}_bench.log').read().strip().splitlines()[-1]); print(d['roofline']['bytes_per_step'])")
  KEY=$(python3 $R/bench.py --workload $W --print-traffic-key)
  EXCL=""; [ $W = nodes64 ] && EXCL="--exclude root_lnl"  # the 64 lnL launches run after the timed steps
  python3 $R/tools/pmc_step.py $OUT/${W}_fetch/run_counter_collection.csv $OUT/${W}_write/run_counter_collection.csv $OUT/${W}_pmc_traffic.json --steps $((P + 2)) --alg-bytes $ALG --key $KEY $EXCL > /dev/null && echo "$W traffic ok"
done
