#!/bin/bash
# SQ counters of the exact-mode protein A/B harness (tools/ab_prot_exact.hip)
# at one size, one rocprofv3 --pmc pass per counter set, summarised per kernel
# (median per dispatch): A = plf_prot_lds_kernel, B = plf_prot_wt_kernel.
#   tools/pmc_ab_prot.sh TAG BINARY SITES
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; BIN=$2; N=$3
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/sq$i -o run --output-format csv -- $R/$BIN $N > $OUT/sq$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
done
for k in plf_prot_lds_kernel plf_prot_wt_kernel; do
  python3 $R/tools/pmc_summary.py $OUT/pmc_$k.json $k $(find $OUT -path "*sq*" -name "*counter_collection.csv") --note "median per dispatch of $k ($BIN $N), tools/pmc_ab_prot.sh"
done
rm -rf $OUT/sq*/
