#!/usr/bin/env python3
"""Probe (not product code): what the node kernel's two small streams -- the
int32 weight read and the uint8 scaler write, 5 B of its 389 B per site --
cost by site count.  One f64 / f32 node call per variant, variants alternating
on the same buffers (median of 5 calls each):
  full       wgt, scaler bytes, scaler sum (the bench's call)
  no-bytes   wgt and sum, no scaler bytes
  no-wgt     scaler bytes and sum, weights = 1 (wgt NULL)
  bare       neither, no sum (the kernel's kSum = false instantiation)
The streaming probe (tools/probes/size_scaling.hip) has neither stream.

  python3 tools/probes/node_streams.py [--sizes 1048576,16777216,67108864,100000000]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402


def case(ctx, tdt, n, calls):
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x1 = torch.empty(16 * n, dtype=tdt, device="cuda")
    x2 = torch.empty_like(x1)
    x3 = torch.empty_like(x1)
    for t in (x1, x2):
        for i in range(0, t.numel(), 1 << 30):
            t[i:i + (1 << 30)].uniform_(generator=g)
    x1.view(n, 16)[0::4] *= 1e-12
    EV = torch.rand(16, dtype=tdt, device="cuda", generator=g)
    L = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    R = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    wgt = torch.ones(n, dtype=torch.int32, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    variants = {"full": (wgt, sc, s), "no-bytes": (wgt, None, s), "no-wgt": (None, sc, s),
                "bare": (None, None, None)}
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    ev = {k: [] for k in variants}
    for k, (w, c, ss) in variants.items():  # warm-up
        ctx.plf_dev(x1, x2, x3, EV, L, R, w, c, ss, stream=st)
    for _ in range(calls):
        for k, (w, c, ss) in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            ctx.plf_dev(x1, x2, x3, EV, L, R, w, c, ss, stream=st)
            e1.record(st)
            ev[k].append((e0, e1))
    torch.cuda.synchronize()
    esz = 8 if tdt == torch.float64 else 4
    out = {"dtype": "f64" if esz == 8 else "f32", "sites": n}
    for k, pairs in ev.items():
        ms = sorted(a.elapsed_time(b) for a, b in pairs)
        med = ms[len(ms) // 2]
        out[k] = {"ms": round(med, 4), "frac_385": round((48 * esz + 1) * n / (med * 1e-3) / 8e12, 4)}
    del x1, x2, x3
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1048576,16777216,67108864,100000000")
    ap.add_argument("--calls", type=int, default=5)
    a = ap.parse_args()
    ctx = plfx.Context(0)
    for n in (int(v) for v in a.sizes.split(",")):
        for tdt in (torch.float64, torch.float32):
            print(json.dumps(case(ctx, tdt, n, a.calls)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
