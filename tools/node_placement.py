#!/usr/bin/env python3
"""Is the f64 node kernel's mid-size trough placement?

At 1.6e7-1.3e8 sites the f64 node line ran 0.66-0.71 of 8 TB/s against 0.75
at 2^20-2^22, and two runs of the same code at 2^24 differed by 8 %
(profiles/r05_node_segments_ab.log).  Here, per size, K fresh sets of
buffers (x1, x2, x3, scaler bytes: separate allocations each, the same
values copied into every set) are timed with the SAME call -- the library's
default mapping, and beside it the one-window and the eight-segment mapping
(contexts made with PLFX_NODE_SEGMENTS=0 / 1) -- calls alternating over
(set, mapping) in one process, so that clock, box and code are common to
every cell:
  * spread ACROSS sets at one mapping = placement (same code, same values,
    other physical pages);
  * spread ACROSS mappings within a set = the mapping.
Each call is timed with HIP events on one stream; the median over `--calls`
per cell.  Scaler sums are checked against the scaler bytes (every 4th site
of x1 x 1e-12 rescales, the host_mem.cpp:199-204 share).  One JSON line per
size.

  python3 tools/node_placement.py [--sizes 16777216,50000000,100000000] [--sets 3] [--calls 7]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402

PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def ctx_with(env):
    old = os.environ.get("PLFX_NODE_SEGMENTS")
    if env is None:
        os.environ.pop("PLFX_NODE_SEGMENTS", None)
    else:
        os.environ["PLFX_NODE_SEGMENTS"] = env
    try:
        return plfx.Context(0)
    finally:
        if old is None:
            os.environ.pop("PLFX_NODE_SEGMENTS", None)
        else:
            os.environ["PLFX_NODE_SEGMENTS"] = old


def case(ctxs, n, nsets, calls):
    tdt = torch.float64
    g = torch.Generator(device="cuda")
    g.manual_seed(97)
    sets = []
    for k in range(nsets):
        b = {key: torch.empty(16 * n, dtype=tdt, device="cuda") for key in ("x1", "x2", "x3")}
        if k == 0:
            for key in ("x1", "x2"):
                t = b[key]
                for i in range(0, t.numel(), 1 << 30):
                    t[i:i + (1 << 30)].uniform_(generator=g)
            b["x1"].view(n, 16)[0::4] *= 1e-12
        else:
            for key in ("x1", "x2"):
                b[key].copy_(sets[0][key])
        b["sc"] = torch.empty(n, dtype=torch.uint8, device="cuda")
        sets.append(b)
    EV = torch.rand(16, dtype=tdt, device="cuda", generator=g)
    L = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    R = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    wgt = torch.ones(n, dtype=torch.int32, device="cuda")
    labels = list(ctxs)
    cells = [(k, lb) for k in range(nsets) for lb in labels]
    s = torch.zeros(len(cells), calls + 1, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    for j, (k, lb) in enumerate(cells):  # warm-up, one call per cell
        b = sets[k]
        ctxs[lb].plf_dev(b["x1"], b["x2"], b["x3"], EV, L, R, wgt, b["sc"], s[j, 0:1], stream=st)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2 * calls)] for _ in cells]
    for c in range(calls):
        for j, (k, lb) in enumerate(cells):
            b = sets[k]
            ev[j][2 * c].record(st)
            ctxs[lb].plf_dev(b["x1"], b["x2"], b["x3"], EV, L, R, wgt, b["sc"], s[j, c + 1:c + 2], stream=st)
            ev[j][2 * c + 1].record(st)
    torch.cuda.synchronize()
    ch = 1 << 26
    flags = sum(int(sets[0]["sc"][i:i + ch].sum(dtype=torch.int64).item()) for i in range(0, n, ch))
    same = all(torch.equal(sets[k]["x3"], sets[0]["x3"]) for k in range(1, nsets))
    sums = [int(v) for v in s.flatten().tolist()]
    ok = same and all(v == flags for v in sums) and flags >= n // 4
    bps = 3 * 16 * 8 + 1
    out = {"dtype": "f64", "sites": n, "sets": nsets, "calls": calls, "bytes_per_site": bps, "frac": {}}
    for j, (k, lb) in enumerate(cells):
        ms = sorted(ev[j][2 * c].elapsed_time(ev[j][2 * c + 1]) for c in range(calls))
        med = ms[len(ms) // 2]
        out["frac"].setdefault(lb, []).append(round(bps * n / (med * 1e-3) / 1e9 / PEAK_GBS, 4))
    for lb in labels:
        v = out["frac"][lb]
        out.setdefault("spread_across_sets", {})[lb] = round(max(v) - min(v), 4)
    out["check"] = "ok" if ok else "MISMATCH"
    for b in sets:
        b.clear()
    del sets, wgt
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16777216,50000000,100000000")
    ap.add_argument("--sets", type=int, default=3)
    ap.add_argument("--calls", type=int, default=7)
    a = ap.parse_args()
    ctxs = {"default": ctx_with(None), "one-window": ctx_with("0"), "8-segments": ctx_with("1")}
    bad = 0
    for n in (int(float(v)) for v in a.sizes.split(",")):
        r = case(ctxs, n, a.sets, a.calls)
        bad += r["check"] != "ok"
        print(json.dumps(r), flush=True)
    for c in ctxs.values():
        c.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
