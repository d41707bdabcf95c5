#!/bin/bash
# Protein (BASELINE configs[4]) measurement session (GPU box, via gpurun from
# the repo root): the protein GPU tests, then bench + rocprofv3 trace + PMC
# traffic (tools/gpu_r02_measure.sh) with a long warm-up (the first ~120
# back-to-back launches of a fresh process run up to 15 % slow, then settle:
# profiles/r02_probe_clock_drift.log), then the stall / LDS counter passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r02p}
cd $R
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_protein.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_protein.log 2>&1 || { tail -30 gpurun_out/$T/pytest_protein.log; exit 1; }
tail -1 gpurun_out/$T/pytest_protein.log
bash tools/gpu_r02_measure.sh $T/protein 20 --workload protein --steps 200 --warmup 300 || exit 1
OUT=$R/gpurun_out/$T/protein
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload protein --steps 10 --warmup 2 --launch bound --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d $OUT/sq$i -o run --output-format csv -- python3 $B > $OUT/sq$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/pmc_stalls.json plf_prot_mfma_kernel $(find $OUT -path "*sq*" -name "*counter_collection.csv") --note "median per dispatch of plf_prot_mfma_kernel (bench --workload protein, 2^18 sites, f64 FMA), tools/gpu_r02_protein.sh"
