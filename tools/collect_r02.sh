#!/bin/bash
# Copy one tools/gpu_r02_full.sh session (gpurun_out/<session>/<workload>/...)
# into profiles/ as <tag>_<workload>_*: the bench line, rocprofv3 kernel stats
# and trace, the PMC records (counter CSVs only for the small workloads) and the
# per-launch / per-step HBM traffic that bench.py reads as roofline.traffic.
#   tools/collect_r02.sh SESSION [TAG]
set -eu
S=${1:?session dir under gpurun_out}; TAG=${2:-r02}
O=gpurun_out/$S; P=profiles
[ -f $O/pytest_gpu.log ] && tail -3 $O/pytest_gpu.log > $P/${TAG}_pytest_gpu.log
for W in node node_f32 protein tree64 nodes512; do
  [ -f $O/$W/bench.log ] || continue
  tail -1 $O/$W/bench.log > $P/${TAG}_${W}_bench.json
  cp $O/$W/trace/run_kernel_stats.csv $P/${TAG}_${W}_kernel_stats.csv
  if [ "$W" != nodes512 ]; then
    cp $O/$W/trace/run_kernel_trace.csv $P/${TAG}_${W}_kernel_trace.csv
    cp $O/$W/fetch/run_counter_collection.csv $P/${TAG}_${W}_pmc_fetch.csv
    cp $O/$W/write/run_counter_collection.csv $P/${TAG}_${W}_pmc_write.csv
  fi
  cp $O/$W/pmc_traffic.json $P/${TAG}_${W}_pmc_traffic.json
done
[ -f $O/node/trace/run_agent_info.csv ] && cp $O/node/trace/run_agent_info.csv $P/${TAG}_agent_info.csv
echo "collected $O into $P/${TAG}_*"
