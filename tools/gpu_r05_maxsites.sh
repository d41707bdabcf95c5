#!/bin/bash
# Round 5: the reference sweep's largest site counts (Makefile:16) in one
# device call and the node kernels' XCD-segmented mapping -- the parity
# tests, the timing tool (default cases, then segmented vs unsegmented by
# size) and a kernel trace of the default cases.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_maxsites
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "sweep_maximum or beyond_2g or xcd_segments" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/max_sites.py > $OUT/max_sites.log 2>&1
rc=$?; echo "max_sites rc=$rc"; cut -c1-400 $OUT/max_sites.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/max_sites.py --ab --sizes 1048576,4194304,16777216,33554432,67108864,134217728,268435456,500000000 > $OUT/max_sites_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cut -c1-300 $OUT/max_sites_ab.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d /tmp/prof/ms -o run --output-format csv -- python3 $R/tools/max_sites.py --calls 3 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cp $(find /tmp/prof/ms -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
head -4 $OUT/kernel_stats.csv | cut -c1-300
