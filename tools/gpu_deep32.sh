set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_deep.log 2>&1 || { tail -40 gpurun_out/pytest_deep.log; exit 1; }
tail -1 gpurun_out/pytest_deep.log
for round in 1 2; do
  for d in f32 f64; do
    for f in 2 3; do
      timeout -k 10 200 python bench.py --workload tree64 --dtype $d --fuse $f --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/deep_bench.log 2>&1 || { tail -20 gpurun_out/deep_bench.log; exit 1; }
      grep '^{' gpurun_out/deep_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $d fuse $f', round(d['value']/1e9,2), 'G sites/s', round(d['roofline']['frac']*100,1), '%', d['check'])"
    done
  done
done
