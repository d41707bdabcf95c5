set -e
mkdir -p gpurun_out/r03s
PLFX_TMP_DEEP_DYN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03s/pytest_tree_dyn.log 2>&1
for r in 1 2; do
  for v in 0 1; do
    for args in "--workload tree64" "--workload tree64 --tips" "--workload tree64 --dtype f32" "--workload tree64 --tips --dtype f32"; do
      tag=$(echo "$args" | tr -d ' -')
      PLFX_TMP_DEEP_DYN=$v timeout -k 10 120 python -u bench.py $args --no-cpu-baseline > gpurun_out/r03s/${tag}_dyn${v}_$r.log 2>&1
    done
  done
done
