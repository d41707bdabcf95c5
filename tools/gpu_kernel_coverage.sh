#!/bin/bash
# The GPU test suite under rocprofv3 --kernel-trace --stats (GPU box, via
# gpurun from the repo root): which kernels it launches
# (tools/kernel_coverage.py reads gpurun_out/cov/run_kernel_stats.csv here).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cov -o run --output-format csv -- \
  python3 -m pytest $R/tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > $R/gpurun_out/cov.log 2>&1
rc=$?
grep -E "passed|failed" $R/gpurun_out/cov.log | tail -1
exit $rc
