#!/usr/bin/env python3
"""HBM traffic of one bench step from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE), for multi-kernel steps (tree64): the PLF kernels' dispatches
(the two fused launches of a step share a total grid size, so they are told
apart by neither name nor grid) are summed per kernel name, corrected as
MI355X_MICROARCH.md's HBM section prescribes (x1024; FETCH_SIZE x2 for 16-B/lane
streaming reads, which these kernels' CLV traffic is), and divided by the
profiled steps (warm-up included).

usage: tools/pmc_step.py FETCH_CSV WRITE_CSV OUT_JSON --steps K --alg-bytes B
  (K = steps profiled incl. warm-up, B = algorithmic bytes per step from the
  bench JSON: bytes_per_site x sites, or roofline.achieved x ms_per_step)
"""
import argparse
import collections
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "amd-versal-phylogenetic-likelihood-function_amd"))
from plfx import codeobj  # noqa: E402
import statistics as st


PLF_KERNELS = ("plf_dna", "root_lnl", "plf_prot", "pmatrix", "prot_tiptip")


def launch_shapes(path, exclude=()):
    """{kernel: [[grid size, workgroup size], ...]} of the PLF dispatches."""
    g = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        nm = r["Kernel_Name"]
        if not nm.startswith(PLF_KERNELS) or nm.startswith(tuple(exclude)):
            continue
        base = nm.split("(")[0].split("<")[0].split("::")[-1]
        g[base].add((int(r["Grid_Size"]), int(r["Workgroup_Size"])))
    return {k: sorted([a, b] for a, b in v) for k, v in g.items()}


def groups(path, name, exclude=()):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != name or not r["Kernel_Name"].startswith(PLF_KERNELS):
            continue
        if r["Kernel_Name"].startswith(tuple(exclude)):
            continue
        g[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--alg-bytes", type=float, required=True)
    ap.add_argument("--exclude", action="append", default=[],
                    help="kernel-name prefix launched outside the timed steps (nodes64: root_lnl)")
    ap.add_argument("--key", default=None, help="bench.py --print-traffic-key of the profiled command")
    a = ap.parse_args()
    fg, wg = groups(a.fetch, "FETCH_SIZE", a.exclude), groups(a.write, "WRITE_SIZE", a.exclude)
    rows, tot = [], 0.0
    for key in sorted(set(fg) & set(wg)):
        f = sum(fg[key]) * 1024 * 2 / a.steps
        w = sum(wg[key]) * 1024 / a.steps
        tot += f + w
        rows.append({"kernel": key, "dispatches": len(fg[key]), "per_step": len(fg[key]) / a.steps,
                     "hbm_read_bytes_per_step": f, "hbm_write_bytes_per_step": w,
                     "fetch_KiB_per_dispatch": sorted(set(round(v) for v in fg[key]))[:8]})
    rec = {"groups": rows, "hbm_bytes_per_step": tot, "algorithmic_bytes_per_step": a.alg_bytes,
           "traffic_over_algorithmic": tot / a.alg_bytes,
           "correction": "FETCH_SIZE x1024 x2, WRITE_SIZE x1024 (MI355X_MICROARCH.md, HBM section)"}
    if a.key:
        rec["key"] = a.key
    # ties the record to the machine code it was counted on (bench.py checks it)
    rec["code"] = codeobj.stamp([r["kernel"] for r in rows])
    # and the dispatch shapes it was counted with (bench.py checks the timed graph's)
    rec["launch"] = launch_shapes(a.fetch, a.exclude)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
