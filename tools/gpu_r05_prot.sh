#!/bin/bash
# Round-5 exact protein pass: the protein GPU tests on the
# rebuilt library (bit-exactness of the trimmed exact kernel), then the three
# builds of tools/time_prot_exact.hip (previous header / ldexp scale select /
# + sched_barrier column pins) alternated three times on one box, then one SQ
# counter pass per build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_prot
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -2 $OUT/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name.log; exit $rc; fi
  return 0
}
cd $R
step pytest_protein 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_protein.py tests/test_gpu_api.py -k "protein or Protein or prot or graph_kernel"
for r in 1 2 3; do
  for v in old ldexp new; do
    step time_${v}_$r 120 ./build/time_prot_exact_$v $v
  done
done
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU -d /tmp/pmc_$v -o run --output-format csv -- $R/build/time_prot_exact_$v $v > $OUT/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/pmc_$v.log; exit 1; }
  cp $(find /tmp/pmc_$v -name "*counter_collection.csv" | head -1) $OUT/pmc_$v.csv
done
echo done
