#!/bin/bash
# Copy one measurement session of tools/measure.sh runs (gpurun_out/<session>/<workload>/...)
# into profiles/ as <tag>_<workload>_*: the bench line, rocprofv3 kernel stats
# (and trace / counter CSVs when they came back) and the HBM traffic record
# that bench.py reads as roofline.traffic.
#   tools/collect_r03.sh SESSION [TAG]
set -eu
S=${1:?session dir under gpurun_out}; TAG=${2:-r03}
O=gpurun_out/$S; P=profiles
[ -f $O/pytest_gpu.log ] && tail -3 $O/pytest_gpu.log > $P/${TAG}_pytest_gpu.log
for W in node node_f32 protein protein_exact protein_f32 tree64 tree64_tips nodes512 prottree64 prottree64_tips; do
  [ -f $O/$W/bench.log ] || continue
  tail -1 $O/$W/bench.log > $P/${TAG}_${W}_bench.json
  cp $O/$W/kernel_stats.csv $P/${TAG}_${W}_kernel_stats.csv
  for f in kernel_trace pmc_fetch pmc_write; do
    [ -f $O/$W/$f.csv ] && [ "$W" != nodes512 ] && cp $O/$W/$f.csv $P/${TAG}_${W}_$f.csv
  done
  cp $O/$W/pmc_traffic.json $P/${TAG}_${W}_pmc_traffic.json
done
[ -f $O/node/agent_info.csv ] && cp $O/node/agent_info.csv $P/${TAG}_agent_info.csv
echo "collected $O into $P/${TAG}_*"
