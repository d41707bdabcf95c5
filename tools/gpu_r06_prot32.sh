#!/bin/bash
# Round 6: the f32 protein FMA grid with two streams in flight (whole blocks
# per CU, rounded up) -- its tests, its stamped PMC traffic record at the new
# launch shape (tools/measure.sh), the line with and without lanes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_prot32
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_protein.py -x -q -k "streams or f32 or fma" --timeout 240 --timeout-method thread > gpurun_out/r06_prot32/pytest.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06_protein_f32 20 --workload protein --dtype f32 > gpurun_out/r06_prot32/measure.log 2>&1 &&
for r in 1 2; do
  for L in 2 1; do
    timeout -k 10 120 python3 bench.py --workload protein --dtype f32 --steps 200 --warmup 300 --no-cpu-baseline --lanes $L > gpurun_out/r06_prot32/l${L}_$r.log 2>&1 || exit 1
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r06_prot32/l${L}_$r.log') if l.startswith('{')][0]
print('f32 protein lanes $L rep $r: frac %.4f  %.2f us/step  check %s  traffic_stale %s' % (d['roofline']['frac'], d['roofline']['event_us_per_step'], d['check'], d['roofline']['traffic_stale']))"
  done
done
rc=$?
tail -1 gpurun_out/r06_prot32/pytest.log
grep -v "^$" gpurun_out/r06_prot32/measure.log | grep -E "traffic|rc=" | cut -c1-200
exit $rc
