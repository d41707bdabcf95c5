#!/bin/bash
# Round 5: the f32 protein FMA kernel with the device-wide tile queue -- the
# previous header's kernel (build/time_prot_f32_old, header copied to
# build/prot_old) vs the current one's static and queued forms
# (build/time_prot_f32_new), alternated twice on one box (tools/time_prot_f32.hip).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_prot32; mkdir -p $OUT
cd $R
for r in 1 2; do
  timeout -k 10 200 ./build/time_prot_f32_old old >> $OUT/time.log 2>&1 || { tail -3 $OUT/time.log; exit 1; }
  timeout -k 10 200 ./build/time_prot_f32_new new >> $OUT/time.log 2>&1 || { tail -3 $OUT/time.log; exit 1; }
done
cat $OUT/time.log
