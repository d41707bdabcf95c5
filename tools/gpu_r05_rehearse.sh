#!/bin/bash
# Round 5: the driver's N > 1 command shape rehearsed on the one-GPU box --
# 2 and 8 ranks over gloo sharing the GPU (bench.py self-launches
# torch.distributed.run), and 1 rank under torch.distributed.run over RCCL at
# the full default size -- to read the timing fields (value from the common
# start instant, wall_barrier_ms_per_step, value_device, skews) and the
# config.nodes512 sub-record.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_rehearse
mkdir -p $OUT
cd $R
show() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s = d["config"].get("nodes512", {})
print(sys.argv[1].split("/")[-1], "n_gpus", d["n_gpus"], "value %.3e" % d["value"], "ms/step %.4f" % d["ms_per_step"],
      "wall_barrier %.4f" % d["wall_barrier_ms_per_step"], "value_device %.3e" % d["value_device"],
      "skew %.1f/%.1f us" % (d["barrier_skew_us"], d["barrier_exit_skew_us"]), d["check"])
if s:
    print("  nodes512", s["nodes_per_rank"], "per rank", "value %.3e" % s["value"], "frac %.3f" % s["frac"],
          "skew %.1f/%.1f us" % (s["barrier_skew_us"], s["barrier_exit_skew_us"]), s["check"], "extra %.1f s" % s["extra_wall_s"])
PY
}
PLFX_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --sites 262144 --nodes 64 > $OUT/gloo2.log 2>&1 || { tail -20 $OUT/gloo2.log; exit 1; }
show $OUT/gloo2.log
PLFX_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 300 python3 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline --sites 262144 --nodes 64 > $OUT/gloo8.log 2>&1 || { tail -20 $OUT/gloo8.log; exit 1; }
show $OUT/gloo8.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/rccl1.log 2>&1 || { tail -20 $OUT/rccl1.log; exit 1; }
show $OUT/rccl1.log
