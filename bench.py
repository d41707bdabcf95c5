#!/usr/bin/env python3
"""bench.py -- PLF sites/s (4-state DNA, fp64) on 1..8 MI355X + % HBM roofline.

Workload (BASELINE.json configs[1]): one inner-node PLF update
(app/src/plf.cpp:19-65 semantics: two 4x4 P x child-CLV matvecs per Gamma
category, element-wise product, EV back-transform, underflow rescale, per-site
scaler byte and weighted scaler sum) over 2^20 sites in fp64 per GPU per step.
A step is one launch of the fused kernel over one node's CLVs, inputs already
resident in HBM.  Steps rotate over R independent buffer sets (R x 389 MiB >
the 256 MiB Infinity Cache) so every step streams from HBM.

Multi-GPU: one process per GPU (torch.distributed.run); every rank evaluates
its own independent inner nodes (the reference's instance split over sites /
nodes, include.h:181-195) with no data-path collective: weak scaling.  After
the timed region one RCCL all-reduce combines the per-rank scaler totals.

Prints ONE JSON line on rank 0 (driver contract), with
  roofline:      algorithmic bytes per launch / average launch duration
                 (HIP events on the launch stream) against 8 TB/s, at SURVEY
                 8(d)'s 385 B/site (x1, x2 read, x3 and the scaler byte
                 written; `achieved_incl_wgt` adds the 4-B weight read); `traffic`
                 = HBM bytes per launch from the committed rocprofv3 PMC pass
                 (profiles/), or null;
  cpu_baseline:  the oracle's OpenMP f64 port on this host's cores over a
                 bounded sample (plus the single-thread port and the reference
                 plf() itself at its own -O0 flags as extra fields).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "amd-versal-phylogenetic-likelihood-function_amd"
sys.path.insert(0, str(PKG))

METRIC = "PLF sites/sec (4-state DNA, fp64) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 20250117


WGT_BYTES = 4  # the kernels also read the int32 site weight for the weighted scaler sum


def bytes_per_site(dtype_bytes):
    # SURVEY 8(d) headline: read x1, x2 (16 values each), write x3 (16 values),
    # write 1 scaler byte -- 385 B in f64.  The 4-byte weight the kernel also
    # reads is reported beside it (roofline.achieved_incl_wgt), not in it.
    return 3 * 16 * dtype_bytes + 1


def coll_device(device):
    """Device for collective tensors: the GPU under RCCL, the CPU under gloo."""
    import torch
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def combine_ranks(wall_ms, dev_ms, got_sum, expect_sum, device, world):
    """Cross-rank reduction of one bench run: MAX of the timed-region wall and
    device times (the driver contract) and ONE all-reduce (RCCL on GPUs, gloo in
    the CPU tests) of the scaler totals.  Returns (wall_ms, dev_ms, check_ok)."""
    import torch
    import torch.distributed as dist

    device = coll_device(device)

    t = torch.tensor([wall_ms, dev_ms], dtype=torch.float64, device=device)
    tot = torch.stack([got_sum.to(device=device, dtype=torch.int64).reshape(()),
                       torch.tensor(expect_sum, dtype=torch.int64, device=device)])
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return float(t[0]), float(t[1]), int(tot[0]) == int(tot[1])


def traffic_key(a):
    """The configuration a committed PMC traffic record belongs to."""
    mode = "exact" if a.exact else "fma"
    fuse = 0 if a.no_fuse else a.fuse
    return f"{a.workload}:{a.dtype}:{mode}:{'tips' if a.tips else 'dense'}:fuse{fuse}:sites{a.sites}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--sites", type=int, default=1 << 20)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--buffer-sets", type=int, default=4)
    ap.add_argument("--fma", action="store_true",
                    help="protein: fused multiply-add mode (the default; f64 runs on the matrix cores)")
    ap.add_argument("--exact", action="store_true",
                    help="protein: plf()'s separate multiply/add (bit-identical to the double loop)")
    ap.add_argument("--fuse", type=int, choices=[0, 1, 2, 3], default=3,
                    help="tree64 schedule (PLFX_FUSE): 3 fused six-level subtrees (dense leaves) "
                         "before 2's, 2 fused three-level subtrees and level pairs, "
                         "1 level pairs only, 0 one launch per level")
    ap.add_argument("--no-fuse", action="store_true", help="same as --fuse 0")
    ap.add_argument("--tips", action="store_true",
                    help="tree64: tips as uint8 state codes (plfx.h section 8) instead of dense CLVs")
    ap.add_argument("--workload", choices=["node", "tree64", "nodes64", "protein"], default="node",
                    help="node: BASELINE configs[1] (headline); tree64: configs[2]; "
                         "nodes64: the per-GPU shard of configs[3]")
    ap.add_argument("--launch", choices=["bound", "checked", "graph"], default="graph",
                    help="bound: pre-validated launcher per buffer set; checked: full "
                         "argument checks per call; graph: steps captured in one HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=4.0,
                    help="wall seconds per CPU-baseline variant (bounded sample)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "r01_pmc_traffic.json"))
    ap.add_argument("--print-traffic-key", action="store_true",
                    help="print the configuration key of PMC traffic records and exit")
    return ap.parse_args()


def cpu_baseline(n_sites, seconds):
    """Oracle (CPU restatement of plf()) timed on this host: OpenMP f64 over
    up to 16 threads (the primary number), 1-thread f64, and the reference's
    own plf() (f32, its -O0 host flags) when oracle/_ref is present."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import numpy as np

    import oracle as O

    threads = min(16, os.cpu_count() or 1)
    d = O.gen_hostmem(n_sites, np.float64, SEED)
    out = (np.empty(16 * n_sites, np.float64), np.empty(n_sites, np.uint8))

    def timed(fn, sites):
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return reps * sites / el, reps

    mt, reps_mt = timed(lambda: O.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"],
                                      threads=threads, out=out), n_sites)
    n1 = min(n_sites, 1 << 18)
    s1 = {k: (v[:16 * n1] if k in ("x1", "x2") else v) for k, v in d.items()}
    out1 = (np.empty(16 * n1, np.float64), np.empty(n1, np.uint8))
    st, _ = timed(lambda: O.plf(s1["x1"], s1["x2"], s1["EV"], s1["left"], s1["right"], s1["wgt"][:n1],
                                out=out1), n1)
    res = {"value": mt, "unit": "sites/s", "cores": threads, "kind": "port",
           "sample": f"{reps_mt} x {n_sites} sites, f64, host_mem input protocol, "
                     f"OpenMP static split, ~{seconds:.0f}s wall",
           "single_thread_port_f64": st}
    if O.ref_lib("O0") is not None:
        f = O.gen_hostmem(1 << 16, np.float32, SEED)
        rt, _ = timed(lambda: O.ref_plf(f["x1"], f["x2"], f["EV"], f["left"], f["right"], f["wgt"]),
                      1 << 16)
        res["reference_plf_O0_f32_1thread"] = rt
        if O.ref_lib("O3") is not None:  # the same sources at -O3 (no -march, no fast-math)
            r3, _ = timed(lambda: O.ref_plf(f["x1"], f["x2"], f["EV"], f["left"], f["right"],
                                            f["wgt"], opt="O3"), 1 << 16)
            res["reference_plf_O3_f32_1thread"] = r3
    return res


def host_buffers_rate(ctx, n_sites, dtype, seconds=2.0):
    """The plf()-shaped entry on host arrays (plfx_plf_f64/f32: H2D -> kernel ->
    D2H, synchronous, pageable numpy buffers as plf()'s callers pass them):
    the PCIe-inclusive rate, reported beside `value`, never as it."""
    import numpy as np

    rng = np.random.default_rng(SEED)
    x1 = rng.random(16 * n_sites).astype(dtype)
    x2 = rng.random(16 * n_sites).astype(dtype)
    x3 = np.empty_like(x1)
    EV, L, R = (rng.random(16).astype(dtype), rng.random(64).astype(dtype),
                rng.random(64).astype(dtype))
    wgt = np.ones(n_sites, np.int32)
    ctx.plf(x1, x2, x3, EV, n_sites, L, R, wgt)  # warm-up (staging buffers)
    reps, t0 = 0, time.perf_counter()
    while True:
        ctx.plf(x1, x2, x3, EV, n_sites, L, R, wgt)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return reps * n_sites / el, reps


class NodeWorkload:
    """BASELINE configs[1]: one inner node of n sites per GPU per step, rotating
    over R buffer sets (R x 389 MiB > the 256 MiB Infinity Cache)."""

    def __init__(self, ctx, a, dev, g, tdt, esz):
        import torch

        n, R = a.sites, max(1, a.buffer_sets)
        self.n, self.R = n, R
        self.EV = torch.rand(16, dtype=tdt, device=dev, generator=g)
        self.left = torch.rand(64, dtype=tdt, device=dev, generator=g)
        self.right = torch.rand(64, dtype=tdt, device=dev, generator=g)
        self.sets = []
        for _ in range(R):
            x1 = torch.rand(n * 16, dtype=tdt, device=dev, generator=g)
            x1.view(-1, 16)[0::4] *= 1e-12  # host_mem.cpp:200-202: every 4th site underflows
            x2 = torch.rand(n * 16, dtype=tdt, device=dev, generator=g)
            self.sets.append(dict(x1=x1, x2=x2, x3=torch.empty_like(x1),
                                  wgt=torch.ones(n, dtype=torch.int32, device=dev),
                                  sc=torch.empty(n, dtype=torch.uint8, device=dev),
                                  s=torch.zeros(1, dtype=torch.int64, device=dev)))
        self.ctx, self.checked = ctx, a.launch == "checked"
        self.bound = [ctx.bind_plf_dev(b["x1"], b["x2"], b["x3"], self.EV, self.left, self.right,
                                       b["wgt"], b["sc"], b["s"]) for b in self.sets]
        self.sites_per_step = n
        self.bytes_per_step = bytes_per_site(esz) * n
        self.bytes_per_site = bytes_per_site(esz)
        self.wgt_bytes_per_step = WGT_BYTES * n
        self.config = {
            "workload": f"DNA 4-state x 4 Gamma cats, 1 inner node per GPU per step, {n} sites, "
                        f"{a.dtype} (BASELINE configs[1])",
            "sites_per_gpu_per_step": n, "nodes_per_gpu_per_step": 1, "buffer_sets": R}

    def step(self, i, sh):
        if self.checked:
            b = self.sets[i % self.R]
            self.ctx.plf_dev(b["x1"], b["x2"], b["x3"], self.EV, self.left, self.right, b["wgt"],
                             b["sc"], b["s"], stream=sh)
        else:
            self.bound[i % self.R](sh)

    def check(self):
        import torch

        # every buffer set's last scaler total is n/4 (every 4th site, wgt = 1)
        return torch.stack([b["s"][0] for b in self.sets]).sum(), self.R * ((self.n + 3) // 4)

    def post(self, world, dev):
        return {}


class Tree64Workload:
    """BASELINE configs[2]: post-order sweep of a 64-taxon balanced tree (63
    inner nodes, levels of 32/16/8/4/2/1 nodes, one batched launch per level)
    over n sites, then the root log-likelihood.  Tips dense U[0,1); P and EV
    x0.25 so magnitudes stay bounded and deep levels underflow."""

    def __init__(self, ctx, a, dev, g, tdt, esz):
        import numpy as np
        import torch

        n = a.sites
        ntips = 64
        self.n, self.ctx = n, ctx
        self.ops = np.array(_balanced_ops(ntips), np.int32)
        nops = self.ops.shape[0]
        self.tips = None
        if a.tips:
            acgt = torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device=dev)
            self.tips = [acgt[torch.randint(0, 4, (n,), device=dev, generator=g)]
                         for _ in range(ntips)] + [None] * nops
            self.clv = [None] * ntips
        else:
            self.clv = [torch.rand(16 * n, dtype=tdt, device=dev, generator=g) for _ in range(ntips)]
        self.clv += [torch.empty(16 * n, dtype=tdt, device=dev) for _ in range(nops)]
        self.pm = torch.rand(nops * 128, dtype=tdt, device=dev, generator=g) * 0.25
        self.EV = torch.rand(16, dtype=tdt, device=dev, generator=g) * 0.25
        self.wgt = torch.ones(n, dtype=torch.int32, device=dev)
        self.sums = torch.zeros(nops, dtype=torch.int64, device=dev)
        self.lnl = torch.zeros(1, dtype=torch.float64, device=dev)
        self.sites_per_step = nops * n
        # per node: read x1, x2, write x3, read wgt (scaler sums, no bytes); + lnL read of the root.
        # With coded tips a tip child reads 1 code byte instead of a CLV.  Fused level pairs:
        # A, B and their parent P in one pass -- 4 child reads + 3 writes + wgt.  Fused
        # three-level subtrees: 7 nodes in one pass -- 8 child reads + 7 writes + wgt.
        clv_b, tip_b = 16 * esz, 1
        leaf = tip_b if a.tips else clv_b
        fuse = 0 if a.no_fuse else a.fuse
        self.bytes_per_site = 3 * clv_b + 4
        if fuse == 3 and not a.tips:  # the whole tree as one six-level subtree
            self.bytes_per_step = ((64 * leaf + 63 * clv_b + 4) + (clv_b + 4)) * n
            sched = "fused six-level subtree: one 63-node pass"
        elif fuse >= 2:  # levels 0-2 as 8 seven-node subtrees, levels 3-5 as one
            self.bytes_per_step = (8 * (8 * leaf + 7 * clv_b + 4) + (15 * clv_b + 4)
                                   + (clv_b + 4)) * n
            sched = "fused three-level subtrees: 9 seven-node passes in 2 launches"
        elif fuse == 1:  # levels (32,16), (8,4), (2,1) as 16 + 4 + 1 triples
            first = 4 * leaf + 3 * clv_b + 4
            self.bytes_per_step = (16 * first + 5 * (7 * clv_b + 4) + (clv_b + 4)) * n
            sched = "fused level pairs: 21 three-node passes in 3 launch groups"
        else:
            first = 2 * leaf + clv_b + 4
            self.bytes_per_step = (32 * first + 31 * (3 * clv_b + 4) + (clv_b + 4)) * n
            sched = "6 level launches"
        tipdesc = "tips as uint8 state codes" if a.tips else "dense tip CLVs"
        self.config = {
            "workload": f"DNA 4-state, 64-taxon balanced tree post-order sweep (63 inner nodes, "
                        f"{sched}) + root lnL, {n} sites, {a.dtype}, {tipdesc} "
                        f"(BASELINE configs[2])",
            "sites_per_gpu_per_step": self.sites_per_step, "nodes_per_gpu_per_step": nops}

    def step(self, i, sh):
        self.ctx.traverse(self.ops, self.clv, self.pm, self.EV, self.n, self.wgt, None, self.sums,
                          stream=sh, tips=self.tips)
        self.ctx.root_lnl(self.clv[-1], self.n, self.lnl, wgt=self.wgt, scaler_sums=self.sums,
                          stream=sh)

    def check(self):
        import torch

        ok = bool(torch.isfinite(self.lnl).all().item()) and int(self.sums.sum().item()) > 0
        return torch.tensor(1 if ok else 0), 1

    def post(self, world, dev):
        import torch
        import torch.distributed as dist

        # each rank holds its own block of n alignment sites (the reference's instance
        # split, include.h:181-195): the tree lnL is the sum over ranks -- one all-reduce
        tot = torch.stack([self.lnl[0], self.sums.sum().to(torch.float64)]).to(coll_device(dev))
        if world > 1:
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        return {"root_lnl_rank0": float(self.lnl.item()), "tree_lnl_all_ranks": float(tot[0]),
                "scaler_events_all_ranks": int(tot[1]),
                "alignment_sites": world * self.n}


class Nodes64Workload:
    """BASELINE configs[3] per-GPU shard: 512 independent inner nodes x n sites
    over 8 GPUs = 64 nodes per GPU per step (two 32-node batched launches).  After
    the timed region every rank evaluates the lnL of its nodes and ONE RCCL
    all-reduce sums the lnL and scaler totals over ranks."""

    def __init__(self, ctx, a, dev, g, tdt, esz):
        import torch

        n = a.sites
        self.n, self.ctx, self.nn = n, ctx, 64
        self.EV = torch.rand(16, dtype=tdt, device=dev, generator=g)
        self.wgt = torch.ones(n, dtype=torch.int32, device=dev)
        self.sums = torch.zeros(self.nn, dtype=torch.int64, device=dev)
        self.nodes = []
        for j in range(self.nn):
            x1 = torch.rand(n * 16, dtype=tdt, device=dev, generator=g)
            x1.view(-1, 16)[0::4] *= 1e-12
            self.nodes.append(dict(
                x1=x1, x2=torch.rand(n * 16, dtype=tdt, device=dev, generator=g),
                x3=torch.empty(n * 16, dtype=tdt, device=dev),
                left=torch.rand(64, dtype=tdt, device=dev, generator=g),
                right=torch.rand(64, dtype=tdt, device=dev, generator=g),
                scaler=torch.empty(n, dtype=torch.uint8, device=dev),
                scaler_sum=self.sums[j:j + 1]))
        self.sites_per_step = self.nn * n
        self.bytes_per_site = bytes_per_site(esz)
        self.bytes_per_step = self.nn * self.bytes_per_site * n
        self.wgt_bytes_per_step = WGT_BYTES * self.nn * n
        self.config = {
            "workload": f"DNA 4-state, 512 independent inner nodes sharded 64 per GPU, {n} sites, "
                        f"{a.dtype} (BASELINE configs[3]); lnL all-reduce after the timed region",
            "sites_per_gpu_per_step": self.sites_per_step, "nodes_per_gpu_per_step": self.nn}

    def step(self, i, sh):
        self.ctx.plf_batch_dev(self.nodes[:32], self.EV, self.n, self.wgt, stream=sh)
        self.ctx.plf_batch_dev(self.nodes[32:], self.EV, self.n, self.wgt, stream=sh)

    def check(self):
        return self.sums.sum(), self.nn * ((self.n + 3) // 4)

    def post(self, world, dev):
        import torch
        import torch.distributed as dist

        lnl = torch.zeros(self.nn, dtype=torch.float64, device=dev)
        for j, nd in enumerate(self.nodes):
            self.ctx.root_lnl(nd["x3"], self.n, lnl[j:j + 1], wgt=self.wgt,
                              scaler_sums=self.sums[j:j + 1])
        tot = torch.stack([lnl.sum(), self.sums.sum().to(torch.float64)]).to(coll_device(dev))
        if world > 1:
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)  # the one lnL all-reduce (RCCL over xGMI)
        return {"lnl_all_nodes_all_ranks": float(tot[0]), "scaler_events_all_ranks": int(tot[1])}


class ProteinWorkload:
    """BASELINE configs[4]: one protein inner node (S=20 states x 4 Gamma
    categories) of n sites (default 2^18) per GPU per step, rotating buffer sets."""

    def __init__(self, ctx, a, dev, g, tdt, esz):
        import torch

        n = a.sites if a.sites != (1 << 20) else (1 << 18)
        R = max(1, a.buffer_sets)
        V = 80
        self.n, self.R, self.ctx, self.fma = n, R, ctx, not a.exact
        self.EV = torch.rand(400, dtype=tdt, device=dev, generator=g) - 0.25
        self.left = torch.rand(1600, dtype=tdt, device=dev, generator=g)
        self.right = torch.rand(1600, dtype=tdt, device=dev, generator=g)
        self.tips = a.tips
        self.sets = []
        for _ in range(R):
            x1 = torch.rand(n * V, dtype=tdt, device=dev, generator=g)
            x1.view(-1, V)[0::4] *= 1e-14
            x2 = torch.rand(n * V, dtype=tdt, device=dev, generator=g)
            codes = None
            if a.tips:  # coded left child: the underflowing sites come from x2 instead
                codes = torch.randint(0, 24, (n,), device=dev, generator=g).to(torch.uint8)
                x2.view(-1, V)[0::4] *= 1e-14
            self.sets.append(dict(x1=x1, x2=x2, x3=torch.empty_like(x1), codes=codes,
                                  wgt=torch.ones(n, dtype=torch.int32, device=dev),
                                  sc=torch.empty(n, dtype=torch.uint8, device=dev),
                                  s=torch.zeros(1, dtype=torch.int64, device=dev)))
        self.sites_per_step = n
        # --tips: the left child is a tip (one code byte per site, plfx.h section 8)
        self.bytes_per_site = (1 if a.tips else V * esz) + 2 * V * esz + 1  # 1921 B f64
        self.bytes_per_step = self.bytes_per_site * n
        self.wgt_bytes_per_step = WGT_BYTES * n
        mode = ('FMA (within 1e-12 of exact)' if esz == 8 else 'FMA') if self.fma else 'exact'
        self.config = {
            "workload": f"Protein 20-state x 4 Gamma cats, 1 inner node per GPU per step, {n} sites, "
                        f"{a.dtype}, {mode}{', tip/inner (coded left child)' if a.tips else ''} "
                        f"(BASELINE configs[4])",
            "sites_per_gpu_per_step": n, "nodes_per_gpu_per_step": 1, "buffer_sets": R}

    def step(self, i, sh):
        b = self.sets[i % self.R]
        if self.tips:
            self.ctx.plf_tips_dev(b["x3"], self.EV, self.n, self.left, self.right, tip1=b["codes"],
                                  x2=b["x2"], wgt=b["wgt"], scaler=b["sc"], scaler_sum=b["s"],
                                  stream=sh, states=20, fma=self.fma)
            return
        self.ctx.plf_dev_gen(b["x1"], b["x2"], b["x3"], self.EV, self.left, self.right, 20,
                             b["wgt"], b["sc"], b["s"], fma=self.fma, stream=sh)

    def check(self):
        import torch

        return torch.stack([b["s"][0] for b in self.sets]).sum(), self.R * ((self.n + 3) // 4)

    def post(self, world, dev):
        return {}


def _balanced_ops(ntips):
    ops, level, nxt = [], list(range(ntips)), ntips
    while len(level) > 1:
        new = []
        for i in range(0, len(level), 2):
            ops.append((nxt, level[i], level[i + 1], len(ops)))
            new.append(nxt)
            nxt += 1
        level = new
    return ops


WORKLOADS = {"node": NodeWorkload, "tree64": Tree64Workload, "nodes64": Nodes64Workload,
             "protein": ProteinWorkload}


def main():
    a = parse()
    if a.print_traffic_key:
        print(traffic_key(a))
        return
    os.environ["PLFX_FUSE"] = "0" if a.no_fuse else str(a.fuse)  # read by plfx_ctx_create
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        sys.exit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    # one process per GPU; LOCAL_RANK folds onto the visible devices so the
    # multi-rank path can be rehearsed on fewer GPUs (PLFX_DIST_BACKEND=gloo)
    ngpu = torch.cuda.device_count()
    local_dev = local % max(ngpu, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        backend = os.environ.get("PLFX_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    import plfx

    ctx = plfx.Context(local_dev)
    tdt = torch.float64 if a.dtype == "f64" else torch.float32
    esz = 8 if a.dtype == "f64" else 4
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    wl = WORKLOADS[a.workload](ctx, a, dev, g, tdt, esz)
    stream = torch.cuda.Stream(dev)          # dedicated launch stream; events on it
    sh = stream.cuda_stream
    torch.cuda.synchronize(dev)

    graph = None
    if a.launch == "graph":
        for i in range(max(a.warmup, 4)):
            wl.step(i, sh)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for i in range(a.steps):
                wl.step(a.warmup + i, stream.cuda_stream)
        torch.cuda.synchronize(dev)

    for i in range(a.warmup):
        wl.step(i, sh)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    if graph is not None:
        with torch.cuda.stream(stream):
            graph.replay()
    else:
        for i in range(a.steps):
            wl.step(a.warmup + i, sh)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    wall_ms = (time.perf_counter() - t0) * 1e3
    dev_ms = e0.elapsed_time(e1)

    got, expect = wl.check()
    wall_ms, dev_ms, check_ok = combine_ranks(wall_ms, dev_ms, got, expect, dev, world)
    extra = wl.post(world, dev)

    if rank == 0:
        per_step_ms = dev_ms / a.steps
        achieved = wl.bytes_per_step / (per_step_ms * 1e-3) / 1e9
        traffic = None
        tp = Path(a.traffic_json)
        if a.workload == "node" and tp.exists():
            try:
                tj = json.loads(tp.read_text())
                if tj.get("sites") == a.sites and tj.get("dtype") == a.dtype:
                    traffic = tj.get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                traffic = None
        # multi-kernel / other workloads: per-step traffic from tools/pmc_step.py,
        # matched on the configuration key and the algorithmic bytes per step
        wtp = {"tree64": "tree_pmc_traffic", "nodes64": "nodes64_pmc_traffic",
               "protein": "protein_pmc_traffic"}.get(a.workload)
        ttp = Path(a.traffic_json).with_name(Path(a.traffic_json).name.replace("pmc_traffic", wtp)) if wtp else None
        if ttp is not None and ttp.exists():
            try:
                tj = json.loads(ttp.read_text())
                if (abs(tj.get("algorithmic_bytes_per_step", 0) - wl.bytes_per_step) < 1
                        and tj.get("key", traffic_key(a)) == traffic_key(a)):
                    traffic = tj.get("hbm_bytes_per_step")
            except (ValueError, OSError):
                traffic = None
        value = world * wl.sites_per_step * a.steps / (wall_ms * 1e-3)
        cfg = dict(wl.config)
        par = (f"alignment sites sharded x{world} (each GPU sweeps the whole tree over its "
               "own site block; one lnL all-reduce after the timed region)"
               if a.workload == "tree64" else
               f"independent nodes x{world} (one process per GPU, no data-path collective)")
        cfg.update(parallelism=par, launch=a.launch, **extra)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "sites/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": wall_ms / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (torch.rand U[0,1) CLVs/P/EV, left CLV x1e-12 on every 4th site, wgt=1)",
            "config": cfg,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_site": wl.bytes_per_site,
                **({"achieved_incl_wgt": (wl.bytes_per_step + wl.wgt_bytes_per_step)
                                         / (per_step_ms * 1e-3) / 1e9,
                    "bytes_per_site_incl_wgt": wl.bytes_per_site + WGT_BYTES}
                   if hasattr(wl, "wgt_bytes_per_step") else {}),
                "bytes_per_step": wl.bytes_per_step,
                "kernel_avg_us": per_step_ms * 1e3,
            },
            "check": "ok" if check_ok else "CHECK_FAILED",
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cb = cpu_baseline(a.sites, a.cpu_seconds)
            if a.workload == "node":
                # the reference host's report rows (timing.h:107-151): its CPU
                # plf() as "Reference" and the speed-ups excluding / including
                # the host<->device transfers
                import numpy as np

                hb, reps = host_buffers_rate(ctx, a.sites, np.float64 if esz == 8 else np.float32)
                out["host_buffers"] = {
                    "value": hb, "unit": "sites/s",
                    "sample": f"{reps} x plfx_plf_{a.dtype}({a.sites} sites) on pageable host arrays"}
                ref = cb.get("reference_plf_O0_f32_1thread")
                if ref:
                    out["speedup_vs_reference_plf"] = {"excluding_pcie": value / ref,
                                                       "including_pcie": hb / ref}
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if not check_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
