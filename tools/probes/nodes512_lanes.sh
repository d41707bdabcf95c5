#!/bin/bash
# Probe session (not product code): configs[3] (512 nodes x 2^20 f64 sites on
# one GPU) as the batched kernel (32 nodes per launch) or one-node launches,
# on one stream or two lanes (bench.py --workload nodes512), alternated.
set -u
mkdir -p gpurun_out/r06_n512
one() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --workload nodes512 --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r06_n512/$name.log 2>&1 || { tail -5 gpurun_out/r06_n512/$name.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_n512/$name.log') if l.startswith('{')][0]
print('$name', '$*', 'frac %.4f  %.3f ms/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'] / 1e3, d['config'].get('lanes'), d['check']))"
}
for rep in 1 2; do
  one b32_l1_$rep --lanes 1
  one b32_l2_$rep
  one b1_l2_$rep --per-launch 1
  one b1_l1_$rep --per-launch 1 --lanes 1
done
