#!/bin/bash
# Size sweep of the bench lines (GPU box, via gpurun from the repo root): node
# f64 / f32 and protein FMA at several alignment lengths, one bench process
# each (no CPU baseline), for DESIGN's per-size table.  Stops at the first
# failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r02s}
mkdir -p $O
cd $R
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 180 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', '%.3e'%d['value'], '%.2f us'%r['kernel_avg_us'], 'frac %.3f'%r['frac'])"
}
for s in 262144 524288 1048576 2097152 4194304 8388608; do
  run f64_$s --sites $s --steps 100 --warmup 20
  run f32_$s --sites $s --dtype f32 --steps 100 --warmup 20
done
for s in 65536 262144 1048576; do
  run prot_$s --workload protein --sites $s --steps 100 --warmup 300
done
