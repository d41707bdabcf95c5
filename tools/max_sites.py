#!/usr/bin/env python3
"""Rate of ONE plfx_plf_dev call at the largest site counts of the reference's
sweep (Makefile:16, ALIGNMENT_SITES up to 1e9): 1e9 sites f32 and 5e8 sites
f64 (the largest sweep point whose three f64 CLVs fit one MI355X: 192 GB of
CLVs, ~197 GB with weights and scaler bytes).  Inputs are U[0,1) on the device
(torch, seeded) with every 4th left-CLV site x1e-12, so exactly the
host_mem.cpp:199-204 share of sites scales; the check is Σ scaler·wgt against
the sum over the per-site scaler bytes.  Correctness at these sizes is asserted
bit-exactly by tests/test_gpu_parity.py::test_plf_dev_reference_sweep_maximum;
this only times it.  One JSON line per case.  --ab: each size also on a
context with the node kernels' XCD-segmented mapping off (PLFX_NODE_SEGMENTS=0),
calls alternating between the two contexts on the same buffers; --variants
adds contexts made with other library env knobs (grid cap, mapping); --sizes
picks other site counts (f64 and f32 at each; f32 alone above 5e8).

  python3 tools/max_sites.py [--calls 5] [--ab] [--sizes 16777216,67108864]
"""
import os
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402

PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def case(ctxs, tdt, n, calls):
    """ctxs: {label: plfx.Context}; their calls alternate, `calls` each."""
    esz = 8 if tdt == torch.float64 else 4
    g = torch.Generator(device="cuda")
    g.manual_seed(97)
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
    labels = list(ctxs)
    s = torch.zeros(len(labels), calls + 1, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    # the inputs were made on torch's current stream, which `st` does not
    # follow: every fill is done before st starts
    torch.cuda.synchronize()
    for j, lb in enumerate(labels):  # warm-up, one call per context
        ctxs[lb].plf_dev(x1, x2, x3, EV, L, R, wgt, sc, s[j, 0:1], stream=st)
    ev = {lb: [torch.cuda.Event(enable_timing=True) for _ in range(2 * calls)] for lb in labels}
    for k in range(calls):
        for j, lb in enumerate(labels):
            ev[lb][2 * k].record(st)
            ctxs[lb].plf_dev(x1, x2, x3, EV, L, R, wgt, sc, s[j, k + 1:k + 2], stream=st)
            ev[lb][2 * k + 1].record(st)
    torch.cuda.synchronize()
    c = 1 << 26
    flags = sum(int(sc[i:i + c].sum(dtype=torch.int64).item()) for i in range(0, n, c))
    sums = [int(v) for v in s.flatten().tolist()]
    ok = all(v == flags for v in sums) and flags >= n // 4
    bps = 3 * 16 * esz + 1
    out = {"dtype": "f64" if esz == 8 else "f32", "sites": n,
           "clv_bytes_gb": round(3 * 16 * esz * n / 1e9, 1), "bytes_per_site": bps}
    for lb in labels:
        ms = sorted(ev[lb][2 * k].elapsed_time(ev[lb][2 * k + 1]) for k in range(calls))
        med = ms[len(ms) // 2]
        gbs = bps * n / (med * 1e-3) / 1e9
        out[lb] = {"ms_per_call_median": round(med, 4), "ms_per_call_min": round(ms[0], 4),
                   "sites_per_s": round(n / (med * 1e-3)), "achieved_GBs": round(gbs, 1),
                   "frac_of_8TBs": round(gbs / PEAK_GBS, 4)}
    out["scaler_sites"] = flags
    out["check"] = "ok" if ok else f"mismatch {sums} vs {flags}"
    del x1, x2, x3, wgt, sc
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--ab", action="store_true")
    ap.add_argument("--sizes", default=None)
    ap.add_argument("--variants", default=None,
                    help="more contexts, 'label:ENV=VAL,...;label2:...' (e.g. PLFX_MAX_BLOCKS, "
                         "PLFX_NODE_SEGMENTS), timed alternating with the default one")
    a = ap.parse_args()
    ctxs = {"default": plfx.Context(0)}
    if a.ab:
        os.environ["PLFX_NODE_SEGMENTS"] = "0"
        ctxs["unsegmented"] = plfx.Context(0)
        del os.environ["PLFX_NODE_SEGMENTS"]
    for spec in (a.variants.split(";") if a.variants else []):
        # label:ENV=VAL,ENV=VAL -- a context made with those library env knobs
        label, _, envs = spec.partition(":")
        kv = dict(e.split("=", 1) for e in envs.split(",") if e)
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        ctxs[label] = plfx.Context(0)
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    if a.sizes:
        cases = []
        for n in (int(v) for v in a.sizes.split(",")):
            if n <= 500_000_000:
                cases.append((torch.float64, n))
            cases.append((torch.float32, n))
    else:
        cases = [(torch.float32, 1_000_000_000), (torch.float64, 500_000_000)]
    bad = 0
    for tdt, n in cases:
        r = case(ctxs, tdt, n, a.calls)
        bad += r["check"] != "ok"
        print(json.dumps(r), flush=True)
    for c in ctxs.values():
        c.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
