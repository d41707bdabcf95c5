#!/bin/bash
# Stall / issue counters of one kernel under a bench command (GPU box, via
# gpurun from the repo root), one rocprofv3 --pmc pass per counter set:
#   tools/pmc_stalls.sh TAG KERNEL_PREFIX "bench args"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; K=$2; ARGS=$3
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py $ARGS --steps 10 --warmup 2 --launch bound --no-cpu-baseline --no-second-region"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/sq$i -o run --output-format csv -- python3 $B > $OUT/sq$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/pmc_stalls.json $K $(find $OUT -path "*sq*" -name "*counter_collection.csv") --note "median per dispatch of $K (bench.py $ARGS), tools/pmc_stalls.sh"
cat $OUT/pmc_stalls.json
