#!/bin/bash
# LDS bank-conflict share of the protein FMA kernel variants (GPU box, via
# gpurun from the repo root): the product (kX3 = 2) and the split-B-read
# variant (kSplitB) in tools/tune_prot.hip, one PMC pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_pmc_splitb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $O/p -o run --output-format csv -- $R/build/tune_prot 262144 3 ${1:-splitB} > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
F=$(find $O/p -name "*counter_collection.csv" | head -1)
python3 - $F <<'PY'
import csv, sys, collections, statistics as st
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "prot_mfma" in r["Kernel_Name"]:
        v[(r["Kernel_Name"][:160], r["Counter_Name"])].append(float(r["Counter_Value"]))
names = sorted({k[0] for k in v})
for nm in names:
    c = st.median(v[(nm, "SQ_LDS_BANK_CONFLICT")]); a = st.median(v[(nm, "SQ_LDS_IDX_ACTIVE")])
    print(f"{c/a:.4f} conflict/active  {nm}")
PY
