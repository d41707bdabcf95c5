#!/bin/bash
# Probe session (not product code): the node kernel's grid cap (PLFX_MAX_BLOCKS)
# against the number of lanes the steps alternate over (tools/probes/node_overlap.py
# s1 = one stream, g2c / gc3 / gc4 = 2 / 3 / 4 lanes through the HIP API).
set -u
mkdir -p gpurun_out/r06_grid
run() {  # name, max_blocks, args...
  local name=$1 mb=$2; shift 2
  PLFX_MAX_BLOCKS=$mb timeout -k 10 100 python3 -u tools/probes/node_overlap.py --steps 20,200 --reps 11 "$@" > gpurun_out/r06_grid/$name.log 2>&1 || exit 1
  echo "== $name: max_blocks $mb $*"; grep -v amdgpu.ids gpurun_out/r06_grid/$name.log
}
run a_1024 1024 --only s1,g2c
run b_512 512 --only g2c
run c_384 384 --only g2c
run d_256 256 --only g2c,gc4
run e_341 341 --only gc3 --sets 6
run f_512_4 512 --only gc4
run g_640 640 --only g2c
run h_512 512 --only g2c
