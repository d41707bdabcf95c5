#!/bin/bash
# Round-5 check on the current tree (via gpurun from the repo root): the GPU
# suite, smoke(), and the driver's default bench command (node line +
# config.nodes512, traffic from the round-5 PMC records checked against the
# timed graph's dispatch).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r05_check}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc wall_s=$(python3 -c "print(round($(date +%s.%N) - $t0, 1))")"
  tail -1 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name.log; exit $rc; fi
  return 0
}
cd $R
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
python3 - <<PY
import json
d = json.loads(open("$OUT/bench_driver.log").read().strip().splitlines()[-1])
r, s = d["roofline"], d["config"]["nodes512"]
print("node", round(d["value"] / 1e9, 3), round(r["frac"], 4), r["traffic"], r["traffic_stale"], r["traffic_note"])
print("nodes512", round(s["value"] / 1e9, 3), round(s["frac"], 4), s.get("traffic"), s.get("traffic_note"), s["check"], round(s["extra_wall_s"], 1))
PY
