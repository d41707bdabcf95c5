#!/bin/bash
# Round 5: configs[4] f64 FMA at 2^18 sites (8 tiles per block at 512 blocks)
# against other grid caps (PLFX_MAX_BLOCKS), 2000 timed steps (settled clock),
# alternated twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_prot_grid; mkdir -p $OUT
cd $R
for round in 1 2; do
  for g in 512 256 384 1024; do
    PLFX_MAX_BLOCKS=$g timeout -k 10 200 python -u bench.py --workload protein --no-cpu-baseline --no-second-region > $OUT/g${g}_$round.log 2>&1 || { tail -3 $OUT/g${g}_$round.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/g${g}_$round.log').read().strip().splitlines()[-1])
print('grid $g round $round frac', round(d['roofline']['frac'],4), 'event_us', round(d['roofline']['event_us_per_step'],2), d['check'])"
  done
done
