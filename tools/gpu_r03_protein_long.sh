#!/bin/bash
# Protein (configs[4]) lines at the default 2000 timed steps (GPU box, via
# gpurun from the repo root): bench f64 FMA / f32 FMA / f64 exact, then the
# rocprofv3 kernel trace + stats of the default line (every dispatch).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03e}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u bench.py --workload protein > $OUT/protein_bench.log 2>&1 || exit 1
tail -1 $OUT/protein_bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload protein --dtype f32 --no-cpu-baseline > $OUT/protein_f32_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload protein --exact --no-cpu-baseline > $OUT/protein_exact_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --workload protein --no-cpu-baseline > $OUT/protein_rocprof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cat | head -4
