#!/bin/bash
# Round 6: the adopted VALU FMA protein kernel -- its parity tests, its
# stamped PMC traffic record (tools/measure.sh), and the default command with
# the config.protein.valu_fma sub-record.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_valu_final
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_protein.py tests/test_gpu_bench.py -x -q --timeout 240 --timeout-method thread -k "valu or workload_lines or f32_with" > gpurun_out/r06_valu_final/pytest.log 2>&1 &&
timeout -k 10 900 bash tools/measure.sh r06_protein_valu 20 --workload protein --valu > gpurun_out/r06_valu_final/measure.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_valu_final/bench_default.json 2> gpurun_out/r06_valu_final/bench_default.err
