# A/B (tuning only, round 3; the PLFX_TMP_PROT_BATCH switch was removed after
# the run, mode 1 adopted, profiles/r03_protein_batch_ab.log): protein tree levels as one launch per node (the
# round-2 path, PLFX_TMP_PROT_BATCH=0) vs batched launches of up to 32 nodes
# (node = blockIdx.y) with each node's full resident grid (1: the nodes' blocks
# follow each other through the co-resident slots) or the resident grid split
# over the nodes (2, the DNA batches' rule); a 64-taxon balanced tree at
# 2^18 sites, f64 FMA / exact and f32 FMA, alternating in one process; root CLV
# and every node's scaler sum compared bit for bit across the modes.
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, 'amd-versal-phylogenetic-likelihood-function_amd')
import plfx  # noqa: E402

S, CAT, V = 20, 4, 80


def balanced_ops(ntips):
    ops, level, nxt = [], list(range(ntips)), ntips
    while len(level) > 1:
        up = []
        for i in range(0, len(level), 2):
            ops.append([nxt, level[i], level[i + 1], len(ops)])
            up.append(nxt)
            nxt += 1
        level = up
    return np.array(ops, np.int32)


ctx = plfx.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ntips = 64
ops = balanced_ops(ntips)
nops = ops.shape[0]
for dt, fma in ((torch.float64, True), (torch.float64, False), (torch.float32, True)):
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    clv = [torch.rand(V * n, dtype=dt, device="cuda", generator=g) for _ in range(ntips)]
    clv += [torch.empty(V * n, dtype=dt, device="cuda") for _ in range(nops)]
    pm = torch.rand(nops * 2 * CAT * S * S, dtype=dt, device="cuda", generator=g) * 0.1
    EV = torch.rand(S * S, dtype=dt, device="cuda", generator=g) - 0.25
    wgt = torch.ones(n, dtype=torch.int32, device="cuda")
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
    times, ref = {0: [], 1: [], 2: []}, None
    for rnd in range(3):
        for mode in (0, 1, 2):
            os.environ["PLFX_TMP_PROT_BATCH"] = str(mode)
            ctx.traverse(ops, clv, pm, EV, n, wgt, None, sums, states=S, fma=fma)
            torch.cuda.synchronize()
            got = (clv[-1].view(torch.int64 if dt == torch.float64 else torch.int32).clone(), sums.clone())
            if ref is None:
                ref = got
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), f"mode {mode} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ctx.traverse(ops, clv, pm, EV, n, wgt, None, sums, states=S, fma=fma)
            e1.record()
            torch.cuda.synchronize()
            times[mode].append(e0.elapsed_time(e1) / reps)
    bps = 3 * V * (8 if dt == torch.float64 else 4) + 1
    for mode, ts in times.items():
        t = sorted(ts)[1]
        print(f"{str(dt)[6:]} {'FMA  ' if fma else 'exact'} mode {mode}: {t:8.3f} ms per sweep "
              f"({nops} nodes, {n * nops / t / 1e6:6.3f} G node-sites/s, "
              f"{bps * n * nops / (t * 1e-3) / 8e12:.3f} of 8 TB/s)  all {[f'{x:.3f}' for x in ts]}",
              flush=True)
print("sums", int(ref[1].sum()))
