#!/bin/bash
# The protein / nodes64 part of tools/gpu_measure.sh on its own (bench line,
# kernel trace, FETCH_SIZE and WRITE_SIZE passes, per-step HBM traffic).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if [ $rc -eq 1 ] && [ "$name" != "pytest_gpu" ]; then exit 1; fi
  return 0
}
cd /tmp && export TMPDIR=/tmp
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
