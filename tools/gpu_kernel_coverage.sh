#!/bin/bash
# The GPU test suite under rocprofv3 --kernel-trace --stats (GPU box, via
# gpurun from the repo root): which kernels it launches
# (tools/kernel_coverage.py reads gpurun_out/cov/run_kernel_stats.csv here).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cov -o run --output-format csv -- \
  python3 -m pytest $R/tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
  > $R/gpurun_out/cov.log 2>&1
rc=$?
# the per-dispatch trace is large (the merge back is capped): the stats suffice
find $R/gpurun_out/cov -name "*kernel_trace.csv" -delete
grep -E "passed|failed" $R/gpurun_out/cov.log | tail -1
exit $rc
