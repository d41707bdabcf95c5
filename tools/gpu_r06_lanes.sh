#!/bin/bash
# Round 6 lanes A/B (via gpurun from the repo root): the bench GPU tests, then
# the driver's command with the default lanes (node / protein steps over 2
# streams) and with --lanes 1 (every step on the launch stream), alternated
# twice on one box; each line's fracs summarised.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_lanes
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
summ() {
  grep '^{' $OUT/$1.log > $OUT/$1.json
  python3 - $OUT/$1.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]; p = c["protein"]
print(sys.argv[1].split("/")[-1], "lanes", c["lanes"], "node %.4f (%.2f us ev, %.2f us wall)" % (
    d["roofline"]["frac"], d["roofline"]["event_us_per_step"], d["ms_per_step"] * 1e3),
    "value %.4g" % d["value"], "nodes512 %.4f tree64 %.4f protein %.4f valu %.4f exact %.4f" % (
    c["nodes512"]["frac"], c["tree64"]["frac"], p["frac"], p["valu_fma"]["frac"], p["exact"]["frac"]),
    "checks", d["check"], c["nodes512"]["check"], c["tree64"]["check"], p["check"], p["valu_fma"]["check"],
    p["exact"]["check"])
PY
}
cd $R
step pytest_bench 600 python3 -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread
for rep in 1 2; do
  step lanes_default_$rep 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  summ lanes_default_$rep
  step lanes_one_$rep 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 1
  summ lanes_one_$rep
done
