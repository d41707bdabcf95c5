#!/bin/bash
# Probe session (not product code): the f32 node kernel's grid cap with two
# lanes (tools/probes/node_overlap.py g2c) and one stream (s1).
set -u
mkdir -p gpurun_out/r06_grid32
for mb in 0 256 1024 0; do
  PLFX_MAX_BLOCKS=$mb timeout -k 10 100 python3 -u tools/probes/node_overlap.py --dtype f32 --steps 20,200 --reps 11 --only s1,g2c > gpurun_out/r06_grid32/mb$mb.log 2>&1 || exit 1
  echo "== f32 max_blocks $mb (0 = default 512)"; grep -v amdgpu.ids gpurun_out/r06_grid32/mb$mb.log
done
