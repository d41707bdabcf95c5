#!/bin/bash
# Round 5: tree64 f64 at each schedule (PLFX_FUSE 3 / 2 / 1) under two CLV
# placements (one allocation per CLV, one slab) on one box: does a schedule
# with fewer concurrent streams hold up where the six-level pass's 127-stream
# pattern is slow?
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_fuse_placement
mkdir -p $OUT
cd $R
for r in 1 2; do
  for pl in sep slab; do
    X=""; [ $pl = slab ] && X="--stagger 256"
    for f in 3 2 1; do
      tag=${pl}_f${f}_$r
      timeout -k 10 120 python3 bench.py --workload tree64 --fuse $f --steps 30 --warmup 5 --no-cpu-baseline $X > $OUT/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/$tag.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'G node-sites/s', round(d['ms_per_step'],3), 'ms/sweep')"
    done
  done
done
