#!/bin/bash
# Round 6: configs[3] as one-node launches over two lanes -- the bench / dist /
# streams GPU tests, the stamped PMC traffic record of nodes512 at its new
# dispatch (tools/measure.sh; the bound launchers' 512 validation calls are
# one extra step), then the lanes A/B of the driver's command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_nodes512
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench.py tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q -k "not parity or streams" --timeout 400 --timeout-method thread > gpurun_out/r06_nodes512/pytest.log 2>&1 &&
EXTRA_STEPS=1 timeout -k 10 900 bash tools/measure.sh r06_nodes512 2 --workload nodes512 --steps 20 --warmup 5 > gpurun_out/r06_nodes512/measure.log 2>&1 &&
bash tools/gpu_r06_lanes.sh > gpurun_out/r06_nodes512/lanes.log 2>&1
rc=$?
tail -3 gpurun_out/r06_nodes512/pytest.log
grep -v "^$" gpurun_out/r06_nodes512/measure.log | cut -c1-200
cat gpurun_out/r06_nodes512/lanes.log
exit $rc
