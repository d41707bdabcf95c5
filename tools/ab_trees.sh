# Same-box A/B of two source trees (run from the repo root on the GPU box):
# the pre-change tree is a git worktree at .old (git worktree add .old <rev>; make -C .old/amd-versal-phylogenetic-likelihood-function_amd).
set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
for round in 1 2; do
  for tree in new old; do
    D=$R; [ $tree = old ] && D=$R/.old
    for W in nodes64 protein node; do
      K=20; [ $W = protein ] && K=100; [ $W = node ] && K=200
      timeout -k 10 200 python $D/bench.py --workload $W --no-cpu-baseline --steps $K --warmup 5 > $OUT/ab_$W.log 2>&1 || exit 1
      python3 -c "import json,sys; d=json.loads(open('$OUT/ab_$W.log').read().strip().splitlines()[-1]); print('$round $tree $W', round(d['value']/1e9,3), 'G sites/s', round(d['roofline']['frac']*100,1), '%')"
    done
  done
done
