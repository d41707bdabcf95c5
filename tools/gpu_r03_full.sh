#!/bin/bash
# Round-3 measurement session (GPU box, via gpurun from the repo root): the GPU
# tests, then bench + rocprofv3 trace + PMC traffic for each BASELINE config
# the bench times (tools/gpu_r03_measure.sh).  Stops at the first failure.
#   tools/gpu_r03_full.sh [SESSION] [WORKLOADS...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03m}; shift || true
W=${@:-tests node node_f32 protein tree64 tree64_tips nodes512}
cd $R
mkdir -p gpurun_out/$T
for w in $W; do
  case $w in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
           tail -1 gpurun_out/$T/pytest_gpu.log ;;
    node) KERNEL=plf_dna_f64_pair_kernel bash tools/gpu_r03_measure.sh $T/node 40 || exit 1 ;;
    node_f32) KERNEL=plf_dna_kernel DTYPE=f32 bash tools/gpu_r03_measure.sh $T/node_f32 40 --dtype f32 || exit 1 ;;
    protein) bash tools/gpu_r03_measure.sh $T/protein 20 --workload protein || exit 1 ;;
    tree64) bash tools/gpu_r03_measure.sh $T/tree64 20 --workload tree64 --steps 50 --warmup 5 || exit 1 ;;
    tree64_tips) bash tools/gpu_r03_measure.sh $T/tree64_tips 20 --workload tree64 --tips --steps 50 --warmup 5 || exit 1 ;;
    nodes512) EXTRA_STEPS=1 bash tools/gpu_r03_measure.sh $T/nodes512 2 --workload nodes512 --steps 10 --warmup 2 || exit 1 ;;
    prottree64) bash tools/gpu_r03_measure.sh $T/prottree64 10 --workload prottree64 --steps 50 --warmup 5 || exit 1 ;;
    prottree64_tips) bash tools/gpu_r03_measure.sh $T/prottree64_tips 10 --workload prottree64 --tips --steps 50 --warmup 5 || exit 1 ;;
    protein_exact) bash tools/gpu_r03_measure.sh $T/protein_exact 20 --workload protein --exact || exit 1 ;;
    protein_f32) bash tools/gpu_r03_measure.sh $T/protein_f32 20 --workload protein --dtype f32 || exit 1 ;;
  esac
done
