#!/bin/bash
# Round 5: is tree64 f64 (dense) slower with the lazy-table context (no 95-MB
# table pool allocated before the CLVs)?  Alternating bench processes on one
# box, lazy vs --eager-tables, plus the coded tree and the node line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_tree_ab
mkdir -p $OUT
cd $R
for r in 1 2 3; do
  for m in lazy eager; do
    X=""; [ $m = eager ] && X="--eager-tables"
    timeout -k 10 120 python3 bench.py --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline $X > $OUT/tree64_${m}_$r.log 2>&1 || { echo "tree64 $m $r failed"; tail -5 $OUT/tree64_${m}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/tree64_${m}_$r.log').read().strip().splitlines()[-1]); print('tree64 $m $r', round(d['value']/1e9,3), round(d['roofline']['frac'],4), round(d['roofline'].get('frac_second_region',0),4))"
  done
done
