#!/bin/bash
# Probe session (not product code): protein nodes over 2 vs 3 lanes (6 buffer
# sets so both divide), FMA / VALU FMA / exact, alternated twice.
set -u
mkdir -p gpurun_out/r06_pl3
one() {  # name, args...
  local name=$1; shift
  timeout -k 10 120 python3 bench.py --workload protein --steps 200 --warmup 300 --buffer-sets 6 --no-cpu-baseline "$@" > gpurun_out/r06_pl3/$name.log 2>&1 || { tail -5 gpurun_out/r06_pl3/$name.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_pl3/$name.log') if l.startswith('{')][0]
print('$name', '$*', 'frac %.4f  %.2f us/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['config']['lanes'], d['check']))"
}
for r in 1 2; do
  for m in "" "--valu" "--exact"; do
    one l2${m}_$r --lanes 2 $m
    one l3${m}_$r --lanes 3 $m
  done
done
