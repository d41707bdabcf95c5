#!/bin/bash
# Round 6: counters of the two occupancy A/Bs,
# one rocprofv3 --pmc pass per counter set, each under its own time limit:
#   deep pass (tools/ab_deep_occ.hip) on the sep-rev placement (index 1, the
#   slow one on the boxes measured), product vs U1 w4 vs U1 w2;
#   exact protein (tools/ab_prot_tiles.hip) at 2^18 sites, product vs the
#   three-tile-group forms.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06_pmc_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/deep$i -o run --output-format csv -- $R/build/ab_deep_occ 20 1 1 > $OUT/deep$i.log 2>&1 || { echo "deep pass $i failed"; tail -5 $OUT/deep$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/prot$i -o run --output-format csv -- $R/build/ab_prot_tiles 262144 > $OUT/prot$i.log 2>&1 || { echo "prot pass $i failed"; tail -5 $OUT/prot$i.log; exit 1; }
done
for k in "2, 512, 0, true, 1>" "1, 512, 0, true, 4>" "1, 512, 0, true, 2>"; do
  tag=$(echo "$k" | tr -dc '0-9')
  python3 $R/tools/pmc_summary.py $OUT/deep_$tag.json "$k" $(find $OUT -path "*deep*" -name "*counter_collection.csv") --note "plf_dna_f64_deep_kernel<6, true, true, $k, sep-rev placement, build/ab_deep_occ 20 1 1"
done
for k in "10, true, 1>" "10, true, 3>" "4, true, 3>" "2, true, 3>"; do
  tag=$(echo "$k" | tr -dc '0-9')
  python3 $R/tools/pmc_summary.py $OUT/prot_$tag.json "$k" $(find $OUT -path "*prot*" -name "*counter_collection.csv") --note "plf_prot_lds_kernel<double, true, *, 0, $k at 2^18 sites, build/ab_prot_tiles 262144"
done
# keep the summaries only (gpurun copies back at most 64 MiB)
rm -rf $OUT/deep[0-9]* $OUT/prot[0-9]*
