#!/bin/bash
# Probe session (not product code): configs[3] over two lanes, the batched
# kernel at 32 / 8 / 2 nodes per launch sharing the resident grid with the
# other lane (plfx_ctx_set_streams reaches plfx_plf_batch_dev) vs one launch
# per node, alternated twice.
set -u
mkdir -p gpurun_out/r06_n512b
one() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --workload nodes512 --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r06_n512b/$name.log 2>&1 || { tail -5 gpurun_out/r06_n512b/$name.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_n512b/$name.log') if l.startswith('{')][0]
print('$name', '$*', 'frac %.4f  %.3f ms/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'] / 1e3, d['config'].get('lanes'), d['check']))"
}
for rep in 1 2; do
  one b32_$rep --per-launch 32
  one b1_$rep --per-launch 1
  one b8_$rep --per-launch 8
  one b2_$rep --per-launch 2
done
