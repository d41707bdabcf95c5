#!/bin/bash
# Round 6: the default bench invocation with its sub-records (nodes512,
# tree64, protein FMA + exact), then the bench's distributed GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_dist.log 2>&1
