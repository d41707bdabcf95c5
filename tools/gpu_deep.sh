# six-level fused subtrees: parity tests per kernel variant, then same-box
# tree64 A/B of PLFX_FUSE 2 vs 3 (the variant knob PLFX_DEEP_VARIANT of the
# tuning runs in profiles/r01_deep.log is gone; VARIANTS="1" repeats the product)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-1}; do
  PLFX_DEEP_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q -m gpu -k six_level --timeout 120 --timeout-method thread > gpurun_out/pytest_deep.log 2>&1 || { tail -40 gpurun_out/pytest_deep.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/pytest_deep.log)"
done
for round in 1 2; do
  for tk in ${TIPS:-dense tips}; do
    t=""; [ $tk = tips ] && t=--tips
    for f in 2 $(for v in ${VARIANTS:-1}; do echo 3:$v; done); do
      fu=${f%%:*}; v=${f##*:}
      PLFX_DEEP_VARIANT=$v timeout -k 10 200 python bench.py --workload tree64 --fuse $fu $t --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/deep_bench.log 2>&1 || { tail -20 gpurun_out/deep_bench.log; exit 1; }
      grep '^{' gpurun_out/deep_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round fuse $f $t', round(d['value']/1e9,2), 'G sites/s', round(d['roofline']['frac']*100,1), '%', d['check'])"
    done
  done
done
