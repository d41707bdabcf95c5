#!/bin/bash
# Round 5: tree64 f64 dense, the round-4 tree (build/r04wt, a git worktree of
# f606ba5 built in place) against the current tree, alternated on one box;
# plus the node line of each (no nodes512) as a box reference.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_tree_ab2
mkdir -p $OUT
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 120 python3 bench.py "$@" > $OUT/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), round(d['roofline']['frac'],4))"
}
for r in 1 2; do
  run r04_tree_$r $R/build/r04wt --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline
  run r05_tree_$r $R --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline
  run r04_tree_bound_$r $R/build/r04wt --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline --launch bound
  run r05_tree_bound_$r $R --workload tree64 --steps 50 --warmup 5 --no-cpu-baseline --launch bound
done
run r04_node $R/build/r04wt --no-cpu-baseline
run r05_node $R --no-cpu-baseline --no-nodes512
