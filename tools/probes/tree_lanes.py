#!/usr/bin/env python3
"""Probe (not product code): configs[2]'s 64-taxon sweep with fewer CLV
streams in flight.  The fused six-level pass keeps 127 CLV streams in flight
and runs 0.64-0.77 of HBM depending on where the CLVs sit;
one-node calls on two lanes keep 6 and run 0.79 (nodes512).  Here the same
tree (bench.Tree64Workload's buffers, 2^20 f64 sites):
  six     one plfx_traverse call, the six-level pass (the bench's sweep)
  three   one call on a PLFX_FUSE=2 context: 8 three-level subtrees in one
          launch, then the top three-level subtree
  sub2    the 8 lower three-level subtrees as 8 traverse calls alternating
          over 2 streams, a join, the top subtree (PLFX_FUSE=2 context)
  sub4    the same over 4 streams
  lvl2    level by level, every node its own call, alternating over 2 streams
          with a join per level (plfx_ctx_set_streams 2)
Device time per sweep (events, median of the reps, variants alternating);
every variant's 63 inner CLVs bit-identical to `six`'s.  The sweep's node-sites
per second and the fraction of 8 TB/s over the six-level pass's bytes
(64 leaf reads + 63 writes + wgt), so the variants compare by sweep time.

  python3 tools/probes/tree_lanes.py [--reps 7] [--sites 1048576] [--stagger BYTES]
"""
import argparse
import os
import statistics as st
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import plfx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--sites", type=int, default=1 << 20)
    ap.add_argument("--stagger", type=int, default=0, help="bench.py --stagger: one slab, CLV j at j x (size + stagger)")
    o = ap.parse_args()
    dev = torch.device("cuda", 0)
    a = bench.parse(["--workload", "tree64", "--sites", str(o.sites), "--stagger", str(o.stagger)])
    ctx = plfx.Context(0, lazy_tables=True)
    os.environ["PLFX_FUSE"] = "2"
    ctx2 = plfx.Context(0, lazy_tables=True)
    del os.environ["PLFX_FUSE"]
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    wl = bench.Tree64Workload(ctx, a, dev, g, torch.float64, 8)
    n, ops = wl.n, wl.ops
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    sums = torch.zeros(len(ops), dtype=torch.int64, device=dev)
    # the lower three-level subtrees: leaves 8s..8s+7 -> ops 4s..4s+3 (level 0),
    # 32+2s, 33+2s (level 1), 48+s (level 2); the top one: ops 56..62
    subs = [np.array([4 * s, 4 * s + 1, 4 * s + 2, 4 * s + 3, 32 + 2 * s, 33 + 2 * s, 48 + s]) for s in range(8)]
    top = np.arange(56, 63)
    levels = [np.arange(0, 32), np.arange(32, 48), np.arange(48, 56), np.arange(56, 60), np.arange(60, 62),
              np.arange(62, 63)]
    sub_sums = [torch.zeros(7, dtype=torch.int64, device=dev) for _ in range(9)]
    op_sums = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(len(ops))]

    def trav(c, idx, sh, s_t):
        c.traverse(ops[idx], wl.clv, wl.pm, wl.EV, n, wl.wgt, None, s_t, stream=sh)

    def run_six(sh):
        trav(ctx, np.arange(len(ops)), sh, sums)

    def run_three(sh):
        trav(ctx2, np.arange(len(ops)), sh, sums)

    def run_sub(L):
        def f(sh):
            main = streams[0]
            ev = torch.cuda.Event()
            ev.record(main)
            for st_ in streams[1:L]:
                st_.wait_event(ev)
            for s in range(8):
                trav(ctx2, subs[s], streams[s % L].cuda_stream, sub_sums[s])
            for st_ in streams[1:L]:
                main.wait_stream(st_)
            trav(ctx2, top, main.cuda_stream, sub_sums[8])
        return f

    def run_lvl2(sh):
        main = streams[0]
        ctx.set_streams(2)
        for lv in levels:
            ev = torch.cuda.Event()
            ev.record(main)
            streams[1].wait_event(ev)
            for j, i in enumerate(lv):
                trav(ctx, np.array([i]), streams[j % 2].cuda_stream, op_sums[i])
            main.wait_stream(streams[1])
        ctx.set_streams(1)

    variants = {"six": run_six, "three": run_three, "sub2": run_sub(2), "sub4": run_sub(4), "lvl2": run_lvl2}
    inner = range(64, 127)
    torch.cuda.synchronize()
    run_six(streams[0].cuda_stream)
    torch.cuda.synchronize()
    want = [wl.clv[j].clone() for j in inner]
    res = {k: [] for k in variants}
    ok = {k: True for k in variants}
    for k, f in variants.items():  # warm-up
        f(streams[0].cuda_stream)
    torch.cuda.synchronize()
    for _ in range(o.reps):
        for k, f in variants.items():
            for j in inner:
                wl.clv[j].zero_()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            f(streams[0].cuda_stream)
            e1.record(streams[0])
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3)
            ok[k] = ok[k] and all(torch.equal(wl.clv[j].view(torch.int64), w.view(torch.int64))
                                  for j, w in zip(inner, want))
    six_bytes = (64 * 128 + 63 * 128 + 4) * n
    for k, v in res.items():
        m = st.median(v)
        print(f"{k:6s} {m:8.1f} us per sweep (min {min(v):8.1f})  {63 * n / (m * 1e-6) / 1e9:6.2f} G node-sites/s  "
              f"six-level bytes / time = {six_bytes / (m * 1e-6) / 8e12:.4f}  bits == six: {ok[k]}", flush=True)
    ctx.close()
    ctx2.close()


if __name__ == "__main__":
    main()
