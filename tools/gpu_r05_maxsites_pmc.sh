#!/bin/bash
# Round 5: HBM traffic of the node kernels at the reference sweep's maxima
# (1e9 sites f32, 5e8 f64, XCD-segmented mapping): the two PMC passes over
# tools/max_sites.py, turned into bytes per launch by tools/pmc_traffic.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05_maxsites_pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d /tmp/prof/msf -o run --output-format csv -- python3 $R/tools/max_sites.py --calls 2 > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d /tmp/prof/msw -o run --output-format csv -- python3 $R/tools/max_sites.py --calls 2 > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 1; }
F=$(find /tmp/prof/msf -name "*counter_collection.csv" | head -1)
W=$(find /tmp/prof/msw -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_traffic.py $F $W $OUT/f64_pmc_traffic.json --sites 500000000 --dtype f64 --kernel plf_dna_f64_pair_kernel > /dev/null
python3 $R/tools/pmc_traffic.py $F $W $OUT/f32_pmc_traffic.json --sites 1000000000 --dtype f32 --kernel plf_dna_kernel > /dev/null
for d in f64 f32; do python3 -c "import json; r=json.load(open('$OUT/${d}_pmc_traffic.json')); print('$d', r['hbm_bytes_per_launch'], r['traffic_over_algorithmic'], r['dispatches'], r.get('launch'))"; done
