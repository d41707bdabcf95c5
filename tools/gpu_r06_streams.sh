#!/bin/bash
# Round 6: the one-node grids sized for the bench's two lanes
# (plfx_ctx_set_streams) -- the tests that cover it, the stamped PMC traffic
# records of the node and protein FMA kernels at their new launch shapes
# (tools/measure.sh), then the lanes A/B of the driver's command
# (tools/gpu_r06_lanes.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_streams
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py -x -q -k "streams or segment or bench or workload or default or corrupt" --timeout 240 --timeout-method thread > gpurun_out/r06_streams/pytest.log 2>&1 &&
KERNEL=plf_dna_f64_pair_kernel SITES=1048576 DTYPE=f64 timeout -k 10 900 bash tools/measure.sh r06_node 20 > gpurun_out/r06_streams/measure_node.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06_protein 20 --workload protein > gpurun_out/r06_streams/measure_protein.log 2>&1 &&
bash tools/gpu_r06_lanes.sh > gpurun_out/r06_streams/lanes.log 2>&1
rc=$?
tail -3 gpurun_out/r06_streams/pytest.log
cat gpurun_out/r06_streams/measure_*.log | grep -v "^$" | cut -c1-200
cat gpurun_out/r06_streams/lanes.log
exit $rc
