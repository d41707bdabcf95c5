#!/bin/bash
# Probe session (not product code): the VALU FMA protein kernel with the
# child's row held in registers for the phase (product: 168 VGPRs, 21 spilled)
# vs read from the LDS tile per 2-column chunk (PLFX_VALU_LDSX=1: 2 spilled),
# the tile prefetch kept; the VALU tests with the switch on; two lanes
# alternated three times, then one stream.
# The PLFX_VALU_LDSX switch exists only in the library built from @d4b0f72 (the A/B
# code was removed after it); run this against a checkout of that commit.
set -u
mkdir -p gpurun_out/r06_ldsx
PLFX_VALU_LDSX=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_protein.py -x -q -k valu --timeout 240 --timeout-method thread > gpurun_out/r06_ldsx/pytest.log 2>&1 || { tail -20 gpurun_out/r06_ldsx/pytest.log; exit 1; }
tail -1 gpurun_out/r06_ldsx/pytest.log
one() {  # name, env value, args...
  local name=$1 ev=$2; shift 2
  PLFX_VALU_LDSX=$ev timeout -k 10 120 python3 bench.py --workload protein --steps 200 --warmup 300 --no-cpu-baseline "$@" > gpurun_out/r06_ldsx/$name.log 2>&1 || { tail -5 gpurun_out/r06_ldsx/$name.log; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_ldsx/$name.log') if l.startswith('{')][0]
print('$name', 'frac %.4f  %.2f us/step  lanes %s  check %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['config']['lanes'], d['check']))"
}
for r in 1 2 3; do
  one valu_reg_$r 0 --valu
  one valu_ldsx_$r 1 --valu
done
one valu_reg_l1 0 --valu --lanes 1
one valu_ldsx_l1 1 --valu --lanes 1
one valu_reg_l1b 0 --valu --lanes 1
one valu_ldsx_l1b 1 --valu --lanes 1
