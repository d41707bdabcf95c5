#!/bin/bash
# Same-box A/B of libplfx builds (GPU box, via gpurun from the repo root):
# each named library in tmp_ab/ (built here beforehand) is put in place of
# plfx/libplfx.so in turn and the same bench command runs on it; the in-tree
# library is restored at the end.
#   tools/ab_libs.sh TAG "bench args" lib1 lib2 ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ARGS=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
LIB=$R/amd-versal-phylogenetic-likelihood-function_amd/plfx/libplfx.so
cp $LIB $OUT/.intree.so
cd $R
for L in "$@"; do
  cp tmp_ab/$L.so $LIB
  timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline > $OUT/$L.log 2>&1
  rc=$?
  echo "$L rc=$rc $(tail -1 $OUT/$L.log | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"]/1e9,4), "G", round(d["ms_per_step"]*1e3,2), "us", "frac", round(r["frac"],4), "2nd", r.get("frac_second_region"))
except Exception as e: print("no line", e)')"
  if [ $rc -ne 0 ]; then cp $OUT/.intree.so $LIB; exit $rc; fi
done
cp $OUT/.intree.so $LIB
