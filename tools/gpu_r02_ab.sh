#!/bin/bash
# A/B harness session (GPU box, via gpurun from the repo root):
#   tools/gpu_r02_ab.sh TAG "binary args" ["binary args" ...]
# runs each prebuilt harness invocation under its own time limit, stops at the
# first failure, and prints the tail of each log.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
i=0
for cmd in "$@"; do
  i=$((i + 1))
  timeout -k 10 240 $cmd > $OUT/run$i.log 2>&1
  rc=$?
  echo "== $cmd rc=$rc"
  tail -14 $OUT/run$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
