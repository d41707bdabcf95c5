#!/usr/bin/env python3
"""Median per dispatch of every counter in one or more rocprofv3 --pmc
counter_collection CSVs, for the dispatches of one kernel (name substring), with
the ratios the DESIGN notes quote (LDS bank-conflict cycles / LDS-active
cycles, instruction-wait / wave cycles, MFMA-busy share).

usage: tools/pmc_summary.py OUT_JSON KERNEL_SUBSTRING CSV [CSV ...] [--note TEXT]
"""
import argparse
import collections
import csv
import json
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("kernel")
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    for path in a.csvs:
        for r in csv.DictReader(open(path)):
            if a.kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {k: st.median(v) for k, v in sorted(vals.items())}
    res["dispatches"] = {k: len(v) for k, v in sorted(vals.items())}

    def ratio(name, num, den):
        if num in res and den in res and res[den]:
            res[name] = res[num] / res[den]

    ratio("lds_bank_conflict_over_lds_active", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")
    ratio("wait_inst_over_wave_cycles", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES")
    res["kernel"] = a.kernel
    res["note"] = a.note
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if "over" in k}))


if __name__ == "__main__":
    main()
