#!/bin/bash
# Round 5: tree64 f64 dense ran 0.65 on this round's boxes (the round-4 tree
# too, tools/gpu_r05_tree_ab2.sh) against 0.77 in round 4.  Hypothesis: the 127
# CLVs of 128 MiB are physically contiguous, so a wave's 127 streams at one
# site offset land on the same HBM channels.  Test: the CLVs carved from one
# slab at staggered offsets, alternated with separate allocations.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_tree_stagger
mkdir -p $OUT
cd $R
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 120 python3 bench.py --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline "$@" > $OUT/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), round(d['roofline']['frac'],4), d['config'].get('root_lnl_rank0'))"
}
for r in 1 2; do
  run sep_$r
  for s in 256 4096 65536 2097152 4352 69888; do run st${s}_$r --stagger $s; done
done
run tips_sep --tips
run tips_st4352 --tips --stagger 4352
