set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
PLFX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 2 > gpurun_out/bench_n2_gloo.log 2>&1 || { tail -20 gpurun_out/bench_n2_gloo.log; exit 1; }
grep '^{' gpurun_out/bench_n2_gloo.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 gloo rehearsal', d['n_gpus'], round(d['value']/1e9,2), 'G sites/s', d['check'])"
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default bench', round(d['value']/1e9,3), 'G sites/s', round(d['roofline']['frac']*100,1), '%', d['check'], 'cpu', d['cpu_baseline']['value'])"
