#!/bin/bash
# Round 5: the tree64 placement probe (tools/probes/tree_placement.hip) and the
# bench's tree64 line with separate / slab CLVs, on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_placement
mkdir -p $OUT
cd $R
timeout -k 10 240 ./build/tree_placement > $OUT/probe.log 2>&1 || { echo probe failed; tail -5 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
for t in sep slab; do
  X=""; [ $t = slab ] && X="--stagger 256"
  timeout -k 10 120 python3 bench.py --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline $X > $OUT/tree64_$t.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/tree64_$t.log').read().strip().splitlines()[-1]); print('tree64 $t', round(d['value']/1e9,3), round(d['roofline']['frac'],4))"
done
