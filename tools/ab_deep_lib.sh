# A/B (same box): tree64 with the HEAD library (tmp_ab/libplfx_head.so) vs the
# working tree's, alternating; restores the working tree's library at the end.
set -e
P=amd-versal-phylogenetic-likelihood-function_amd/plfx
mkdir -p gpurun_out/r03t
cp $P/libplfx.so /tmp/libplfx_new.so
trap 'cp /tmp/libplfx_new.so $P/libplfx.so' EXIT
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then cp tmp_ab/libplfx_head.so $P/libplfx.so; else cp /tmp/libplfx_new.so $P/libplfx.so; fi
    for args in "--workload tree64" "--workload tree64 --dtype f32"; do
      tag=$(echo "$args" | tr -d ' -')
      timeout -k 10 120 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03t/${tag}_${v}_$r.log 2>&1
      PLFX_TMP_DEEP_DYN=1 timeout -k 10 120 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03t/${tag}_${v}dyn_$r.log 2>&1
    done
  done
done
