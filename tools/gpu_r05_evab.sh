#!/bin/bash
# Round 5: region events created inside vs before the timed region (needs bench_prev.py = git show <rev>:bench.py at the repo root)
set -u
mkdir -p gpurun_out/r05_evab
for r in 1 2 3 4; do
  for b in bench_prev bench; do
    timeout -k 10 120 python -u $b.py --steps 20 --warmup 5 --no-cpu-baseline --no-nodes512 --no-second-region > gpurun_out/r05_evab/${b}_$r.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/r05_evab/${b}_$r.log').read().strip().splitlines()[-1])
print('$b', $r, round(d['value']/1e9,3), round(d['value_device']/1e9,3), 'gap', round(d['value_device']/d['value']-1,4))"
  done
done
