#!/bin/bash
# Copy one tools/gpu_measure.sh session's outputs from gpurun_out/ into
# profiles/ under the round tag (default r01), the files bench.py and
# profiles/README.md refer to.
set -eu
TAG=${1:-r01}
O=gpurun_out; P=profiles
tail -1 $O/bench.log > $P/${TAG}_bench.json
cp $O/prof_trace/run_kernel_stats.csv $P/${TAG}_kernel_stats.csv
cp $O/prof_trace/run_kernel_trace.csv $P/${TAG}_kernel_trace.csv
cp $O/prof_trace/run_agent_info.csv $P/${TAG}_agent_info.csv
cp $O/prof_fetch/run_counter_collection.csv $P/${TAG}_pmc_fetch.csv
cp $O/prof_write/run_counter_collection.csv $P/${TAG}_pmc_write.csv
cp $O/pmc_traffic.json $P/${TAG}_pmc_traffic.json
tail -3 $O/pytest_gpu.log > $P/${TAG}_pytest_gpu.log
tail -1 $O/tree_bench.log > $P/${TAG}_tree_bench.json
cp $O/tree_trace/run_kernel_stats.csv $P/${TAG}_tree_kernel_stats.csv
cp $O/tree_trace/run_kernel_trace.csv $P/${TAG}_tree_kernel_trace.csv
cp $O/tree_fetch/run_counter_collection.csv $P/${TAG}_tree_pmc_fetch.csv
cp $O/tree_write/run_counter_collection.csv $P/${TAG}_tree_pmc_write.csv
cp $O/tree_pmc_traffic.json $P/${TAG}_tree_pmc_traffic.json
for W in protein nodes64; do
  [ -f $O/${W}_bench.log ] || continue
  tail -1 $O/${W}_bench.log > $P/${TAG}_${W}_bench_session.json
  cp $O/${W}_trace/run_kernel_stats.csv $P/${TAG}_${W}_kernel_stats.csv
  cp $O/${W}_fetch/run_counter_collection.csv $P/${TAG}_${W}_pmc_fetch.csv
  cp $O/${W}_write/run_counter_collection.csv $P/${TAG}_${W}_pmc_write.csv
  cp $O/${W}_pmc_traffic.json $P/${TAG}_${W}_pmc_traffic.json
done
echo "collected into $P/${TAG}_*"
