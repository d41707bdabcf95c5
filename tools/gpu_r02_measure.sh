#!/bin/bash
# Measurement session (GPU box, via gpurun from the repo root): for one bench
# configuration, the bench line, a rocprofv3 kernel trace + stats of the same
# command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE; they do not fit in
# one pass on gfx950) turned into HBM bytes.
#   [KERNEL=name SITES=n DTYPE=f64] tools/gpu_r02_measure.sh TAG PMC_STEPS [bench args...]
# KERNEL set: one kernel per step (the node workloads), traffic = median per
# dispatch of that kernel (tools/pmc_traffic.py); else per step over every
# PLF kernel of the profiled steps (tools/pmc_step.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; P=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -1 $OUT/$name.log | cut -c1-1500
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
cd $R
step bench 300 python -u $R/bench.py "$@"
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline
step fetch 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --steps $P --warmup 2 --launch bound
step write 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- python3 $R/bench.py "$@" --no-cpu-baseline --steps $P --warmup 2 --launch bound
ALG=$(python3 -c "import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['roofline']['bytes_per_step'])")
KEY=$(python3 $R/bench.py "$@" --print-traffic-key)
FCSV=$(find $OUT/fetch -name "*counter_collection.csv" | head -1)
WCSV=$(find $OUT/write -name "*counter_collection.csv" | head -1)
if [ -n "${KERNEL:-}" ]; then
  python3 $R/tools/pmc_traffic.py $FCSV $WCSV $OUT/pmc_traffic.json --sites ${SITES:-1048576} --dtype ${DTYPE:-f64} --kernel $KERNEL > /dev/null
  python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json')); print('traffic', d['hbm_bytes_per_launch'], d['traffic_over_algorithmic'])"
else
  python3 $R/tools/pmc_step.py $FCSV $WCSV $OUT/pmc_traffic.json --steps $((P + 2 + ${EXTRA_STEPS:-0})) --alg-bytes $ALG --key $KEY --exclude root_lnl > /dev/null
  python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json')); print('traffic', d['hbm_bytes_per_step'], d['traffic_over_algorithmic'])"
fi
find $OUT/trace -name "*kernel_stats.csv" -exec head -5 {} \;
