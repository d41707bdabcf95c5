#!/bin/bash
# Round 5: protein and node bench lines with 1 vs 2-4 rotating buffer sets (no
# effect on the rate; profiles/r05_protein_sizes.log context).
set -u
OUT=gpurun_out/r05_sets; mkdir -p $OUT
for spec in "protein 1048576 4" "protein 1048576 1" "protein 4194304 2" "protein 4194304 1" "protein 262144 4" "protein 262144 1" "node 4194304 4" "node 4194304 1" "node 1048576 1"; do
  set -- $spec
  timeout -k 10 200 python -u bench.py --workload $1 --sites $2 --buffer-sets $3 --steps 20 --warmup 3 --no-cpu-baseline --no-second-region --no-nodes512 > $OUT/$1_$2_$3.log 2>&1 || { tail -3 $OUT/$1_$2_$3.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/$1_$2_$3.log').read().strip().splitlines()[-1])
print('$1 $2 sets=$3', 'frac', round(d['roofline']['frac'],3), 'event_us', round(d['roofline']['event_us_per_step'],1))"
done
