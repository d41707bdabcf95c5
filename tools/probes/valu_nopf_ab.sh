#!/bin/bash
# Probe session (not product code): the VALU protein kernels (FMA and exact)
# with the next child tile in flight in registers (product: 168 VGPRs, 21-23
# spilled) vs fetched right before use (PLFX_VALU_NOPF=1: 142-164 VGPRs, no
# spill), two lanes, 2^18 sites, 200 steps after 300 warm-up, alternated 3x.
# The PLFX_VALU_NOPF switch exists only in the library built from @95468ac (the A/B
# code was removed after it); run this against a checkout of that commit.
set -u
mkdir -p gpurun_out/r06_nopf
one() {  # name, env value, args...
  local name=$1 ev=$2; shift 2
  PLFX_VALU_NOPF=$ev timeout -k 10 120 python3 bench.py --workload protein --steps 200 --warmup 300 --no-cpu-baseline "$@" > gpurun_out/r06_nopf/$name.log 2>&1 || { tail -5 gpurun_out/r06_nopf/$name.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_nopf/$name.log') if l.startswith('{')][0]
print('$name', 'frac %.4f  %.2f us/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['config']['lanes'], d['check']))"
}
for r in 1 2 3; do
  one valu_pf_$r 0 --valu
  one valu_nopf_$r 1 --valu
  one exact_pf_$r 0 --exact
  one exact_nopf_$r 1 --exact
done
one valu_pf_l1 0 --valu --lanes 1
one valu_nopf_l1 1 --valu --lanes 1
one exact_pf_l1 0 --exact --lanes 1
one exact_nopf_l1 1 --exact --lanes 1
