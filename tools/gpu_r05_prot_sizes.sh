#!/bin/bash
# Round 5: the protein node lines by site count (does the one-window stride
# lose HBM rate on long protein CLVs as it does for DNA, DESIGN 3.2a?).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_prot_sizes
mkdir -p $OUT
cd $R
# steps: a timed region of ~180-200 ms each, past the post-idle clock dip
# (a 10-step region at 2^18-2^22 sites sits inside it: r05 first pass)
for spec in "f64 262144 4 2000" "f64 1048576 4 500" "f64 4194304 2 150" "f64 16777216 1 40" "f64 33554432 1 20" "f32 262144 4 4000" "f32 1048576 4 1000" "f32 16777216 1 80" "f32 67108864 1 20"; do
  set -- $spec
  timeout -k 10 240 python -u bench.py --workload protein --dtype $1 --sites $2 --buffer-sets $3 --steps $4 --warmup 3 --no-cpu-baseline --no-second-region > $OUT/p_$1_$2.log 2>&1
  rc=$?
  python3 -c "
import json,sys
d=json.loads(open('$OUT/p_$1_$2.log').read().strip().splitlines()[-1])
print('$1', $2, 'value', round(d['value']/1e9,3), 'frac', round(d['roofline']['frac'],3), 'event_us', round(d['roofline']['event_us_per_step'],1), d.get('check'))" || true
  [ $rc -ne 0 ] && { tail -5 $OUT/p_$1_$2.log; exit $rc; }
done
exit 0
