#!/usr/bin/env python3
"""Per-size kernel durations of a `bench.py --sweep` kernel trace: the DNA f64
node kernel's dispatches grouped by grid size (one grid per site count), with
the median and minimum duration.

usage: tools/sweep_kernels.py KERNEL_TRACE_CSV"""
import collections
import csv
import statistics as st
import sys

g = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "plf_dna_f64_pair_kernel" not in r["Kernel_Name"]:
        continue
    grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    g[grid].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'grid threads':>12} {'dispatches':>10} {'median us':>10} {'min us':>8}")
for grid in sorted(g):
    v = g[grid]
    print(f"{grid:>12} {len(v):>10} {st.median(v):>10.2f} {min(v):>8.2f}")
