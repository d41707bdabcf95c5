#!/usr/bin/env python3
"""Per-dispatch PMC series: every dispatch of one kernel (name substring) from
rocprofv3 --pmc counter_collection CSVs under DIR, in dispatch order, one line
per dispatch with each counter's value (summed over its dimensions).  Run on
the GPU box next to the profile so that only this summary travels back.

usage: tools/pmc_series.py DIR KERNEL_SUBSTRING
"""
import collections
import csv
import sys
from pathlib import Path


def main():
    root, kern = Path(sys.argv[1]), sys.argv[2]
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for path in sorted(root.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            if kern not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"][:60]
    if not rows:
        print(f"no dispatch of {kern!r} under {root}")
        return
    cols = sorted({c for v in rows.values() for c in v})
    print("dispatch " + " ".join(cols))
    for d in sorted(rows):
        print(f"{d} " + " ".join(f"{rows[d][c]:.0f}" for c in cols))


if __name__ == "__main__":
    main()
