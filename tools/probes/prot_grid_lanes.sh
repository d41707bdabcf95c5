#!/bin/bash
# Probe session (not product code): the protein node kernels' grid cap
# (PLFX_MAX_BLOCKS) with the bench's two lanes and with one stream, 2^18 sites,
# 200 timed steps after 300 warm-up ones (bench.py --workload protein).
set -u
mkdir -p gpurun_out/r06_pgrid
one() {  # mode args, max_blocks, lanes
  local mode=$1 mb=$2 L=$3
  local extra=""
  [ "$mode" = valu ] && extra="--valu"
  [ "$mode" = exact ] && extra="--exact"
  PLFX_MAX_BLOCKS=$mb timeout -k 10 120 python3 bench.py --workload protein $extra --steps 200 --warmup 300 \
      --no-cpu-baseline --lanes $L > gpurun_out/r06_pgrid/${mode}_${mb}_$L.log 2>&1 || exit 1
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/r06_pgrid/${mode}_${mb}_$L.log') if l.startswith('{')][0]
print('$mode max_blocks $mb lanes $L: frac %.4f  %.2f us/step  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['check']))"
}
for rep in 1 2; do
  for mb in 0 256; do one fma $mb 2; done
  one fma 0 1
  for mb in 0 384 256 512; do one valu $mb 2; done
  one valu 0 1
  for mb in 0 384 256 512; do one exact $mb 2; done
done
