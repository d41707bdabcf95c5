# PMC passes on the protein bench (tuning only): stall/issue counters of the matrix-core kernel.
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_prot
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload protein --steps 10 --warmup 2 --launch bound --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $B > $OUT/p$i.log 2>&1 || exit 1
done
echo ok
