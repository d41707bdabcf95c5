#!/usr/bin/env python3
"""Per-kernel, per-launch-shape summary of a rocprofv3 kernel-trace CSV.

The driver's default command launches the headline node kernel for the
timed region AND, through the host-array leg (plfx_plf_f64 in chunks) and the
CPU-baseline checks, at other grid sizes, so the --stats average of a kernel
mixes launches of different sizes.  This groups the plfx dispatches by
(kernel, grid, workgroup) and prints count / average / min / max duration,
and -- for the longest run of back-to-back dispatches of one shape with no
other dispatch between them (the timed graph's replay; the host-array leg's
launches sit between copy blits; a host synchronisation's idle gap also ends a
run) -- the average over that run alone, and the
run's span (first start to last end) per dispatch, the per-step time when
dispatches overlap (bench.py lanes).  One JSON document.

  python3 tools/trace_by_grid.py KERNEL_TRACE_CSV [OUT_JSON]
"""
import collections
import csv
import json
import statistics as st
import sys


def main():
    path = sys.argv[1]
    def ours(name):  # full (--stats) or truncated (trace) kernel names
        base = name.replace("void ", "").replace("plfx::dev::", "")
        return base.startswith(("plf_", "root_lnl", "scaler_sum", "pmat", "tiptip", "prot_"))

    every = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    pos = {id(r): i for i, r in enumerate(every)}  # position among ALL dispatches (blits included)
    rows = [r for r in every if ours(r["Kernel_Name"])]
    groups = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("plfx::dev::", "")
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        groups[(name, grid, wg)].append(r)
    out = []
    for (name, grid, wg), rs in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
        # the longest run of back-to-back dispatches of this shape with nothing else
        # between them (no blit, no other kernel): the replayed graph of the timed
        # region, not the host-array leg's launches between its copies
        ids = [pos[id(r)] for r in rs]

        def span_of(run):
            # first start to last end: per dispatch, the per-step time when the
            # bench's lanes keep two dispatches in flight (each then lasts ~2x
            # it); equal to the run's average when they run one after another
            return (max(int(rs[i]["End_Timestamp"]) for i in run)
                    - min(int(rs[i]["Start_Timestamp"]) for i in run)) / 1e3

        # a run ends at another dispatch between two of this shape, or at an
        # idle gap over 20 us with none of them in flight (a host
        # synchronisation: the bench's warm-up, its region, its second region)
        runs, cur = [], [0]
        busy = int(rs[0]["End_Timestamp"])  # the current run's latest end
        for i in range(1, len(ids)):
            start, end = int(rs[i]["Start_Timestamp"]), int(rs[i]["End_Timestamp"])
            if ids[i] == ids[i - 1] + 1 and start - busy <= 20000:
                cur.append(i)
                busy = max(busy, end)
            else:
                runs.append(cur)
                cur, busy = [i], end
        runs.append(cur)
        # the longest run; among equally long ones the densest (a run that
        # spans host synchronisations is not the replayed graph)
        best = min(runs, key=lambda r: (-len(r), span_of(r)))
        run = [d[i] for i in best]
        span = span_of(best)
        out.append({"kernel": name, "grid": grid, "workgroup": wg, "dispatches": len(d),
                    "avg_us": round(st.mean(d), 3), "min_us": round(min(d), 3), "max_us": round(max(d), 3),
                    "longest_consecutive_run": len(run), "run_avg_us": round(st.mean(run), 3),
                    "run_span_us_per_dispatch": round(span / len(run), 3),
                    # every run of at least 10: [dispatches, span per dispatch]
                    # (the bench's warm-up, timed region and second region)
                    "runs": [[len(r), round(span_of(r) / len(r), 3)] for r in runs if len(r) >= 10]})
    doc = {"trace": path, "groups": out}
    s = json.dumps(doc, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
