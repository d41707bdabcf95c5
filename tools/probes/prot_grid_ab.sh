#!/bin/bash
# Probe session (not product code): the protein FMA node with two lanes at the
# product's 256-block grid (plfx_ctx_set_streams 2) vs 512 blocks
# (PLFX_MAX_BLOCKS=512), alternated three times on one box; then the same
# with --lanes 1 at 512 (the single-stream default).
set -u
mkdir -p gpurun_out/r06_pab
one() {  # name, max_blocks, args...
  local name=$1 mb=$2; shift 2
  PLFX_MAX_BLOCKS=$mb timeout -k 10 120 python3 bench.py --workload protein --steps 200 --warmup 300 --no-cpu-baseline "$@" > gpurun_out/r06_pab/$name.log 2>&1 || exit 1
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_pab/$name.log') if l.startswith('{')][0]
print('$name', 'max_blocks $mb $*', 'frac %.4f  %.2f us/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['config']['lanes'], d['check']))"
}
for r in 1 2 3; do
  one g256_$r 0
  one g512_$r 512
done
one one_$r 0 --lanes 1
