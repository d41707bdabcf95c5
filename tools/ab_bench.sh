# Same-box A/B of bench.py workloads between this tree and the pre-change tree
# at .old (git worktree add .old <rev>; make -C .old/amd-versal-phylogenetic-likelihood-function_amd).
# Usage (GPU box, repo root): bash tools/ab_bench.sh "<bench args>" [rounds]
set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
ARGS=$1; ROUNDS=${2:-2}
for round in $(seq 1 $ROUNDS); do
  for tree in new old; do
    D=$R; [ $tree = old ] && D=$R/.old
    timeout -k 10 200 python $D/bench.py $ARGS --no-cpu-baseline > $OUT/ab_bench.log 2>&1 || { tail -5 $OUT/ab_bench.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/ab_bench.log').read().strip().splitlines()[-1]); print('$round $tree', round(d['value']/1e9,3), 'G sites/s', round(d['roofline']['frac']*100,1), '%', round(d['roofline']['kernel_avg_us'],1), 'us')"
  done
done
