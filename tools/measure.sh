#!/bin/bash
# Measurement of one bench configuration (GPU box, via gpurun from the repo
# root; round 3's tools/gpu_r03_measure.sh, kept as the tool that makes the
# code-stamped PMC traffic records bench.py reads): the bench line, a rocprofv3 kernel trace + stats of the same
# command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE; they do not fit in
# one pass on gfx950) turned into HBM bytes.  rocprofv3 writes under /tmp;
# only the stats, the traffic record and (when small) the trace and counter
# CSVs are copied to gpurun_out/<TAG>.
#   [KERNEL=name SITES=n DTYPE=f64 EXTRA_STEPS=k] tools/measure.sh TAG PMC_STEPS [bench args...]
# KERNEL set: one kernel per step (the node workloads), traffic = median per
# dispatch of that kernel (tools/pmc_traffic.py); else per step over every
# PLF kernel of the profiled steps (tools/pmc_step.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; P=$2; shift 2
OUT=$R/gpurun_out/$TAG
TMPP=/tmp/prof/$TAG
mkdir -p $OUT $TMPP
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -1 $OUT/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
small() {  # copy a file to OUT if it is under 8 MB
  [ -f "$1" ] && [ $(stat -c %s "$1") -lt 8000000 ] && cp "$1" "$2"
  return 0
}
cd $R
step bench 400 python -u $R/bench.py "$@"
cd /tmp && export TMPDIR=/tmp
step trace 400 rocprofv3 --kernel-trace --stats -T -d $TMPP/trace -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --no-nodes512 --no-tree64 --no-protein
step fetch 400 rocprofv3 --pmc FETCH_SIZE -T -d $TMPP/fetch -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --no-nodes512 --no-tree64 --no-protein --no-second-region --steps $P --warmup 2 --launch bound
step write 400 rocprofv3 --pmc WRITE_SIZE -T -d $TMPP/write -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --no-nodes512 --no-tree64 --no-protein --no-second-region --steps $P --warmup 2 --launch bound
ALG=$(python3 -c "import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['roofline']['bytes_per_step'])")
KEY=$(python3 $R/bench.py "$@" --print-traffic-key)
FCSV=$(find $TMPP/fetch -name "*counter_collection.csv" | head -1)
WCSV=$(find $TMPP/write -name "*counter_collection.csv" | head -1)
if [ -n "${KERNEL:-}" ]; then
  python3 $R/tools/pmc_traffic.py $FCSV $WCSV $OUT/pmc_traffic.json --sites ${SITES:-1048576} --dtype ${DTYPE:-f64} --kernel $KERNEL > /dev/null
  python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json')); print('traffic', d['hbm_bytes_per_launch'], d['traffic_over_algorithmic'])"
else
  python3 $R/tools/pmc_step.py $FCSV $WCSV $OUT/pmc_traffic.json --steps $((P + 2 + ${EXTRA_STEPS:-0})) --alg-bytes $ALG --key $KEY --exclude root_lnl > /dev/null
  python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json')); print('traffic', d['hbm_bytes_per_step'], d['traffic_over_algorithmic'])"
fi
cp $(find $TMPP/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
small "$(find $TMPP/trace -name "*kernel_trace.csv" | head -1)" $OUT/kernel_trace.csv
small "$(find $TMPP/trace -name "*agent_info.csv" | head -1)" $OUT/agent_info.csv
small "$FCSV" $OUT/pmc_fetch.csv
small "$WCSV" $OUT/pmc_write.csv
head -5 $OUT/kernel_stats.csv
rm -rf $TMPP
