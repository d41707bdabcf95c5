"""nodes_sched.py -- probe (not product code): nodes512 (BASELINE configs[3])
at N = 1 with two launch schedules over the same 512 nodes:

  A  consecutive: launch g = nodes 32g .. 32g+31 (allocation order; round 2)
  B  interleaved: launch g = nodes g, g+16, g+32, ... (every launch mixes the
     allocation regions)

tools/probes/nodes_groups.py showed a slow launch group is slow only as a
whole: each of its nodes alone runs like any other node, half of it plus half
of a fast group runs fast, and shifting the nodes' relative alignment by up to
2 MiB changes nothing.  So the cost is tied to which allocations stream at the
same time.  Run under rocprofv3 --pmc for TLB (TCP_UTCL1_*) and DRAM-credit
(TCC_EA0_*) counters per dispatch; dispatch order: R rounds of A's 16
launches, then R rounds of B's.

  python tools/probes/nodes_sched.py [rounds=3] > gpurun_out/nodes_sched.log
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402

SEED = 20250117


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    N, n = 512, 1 << 20
    dev = torch.device("cuda", 0)
    ctx = plfx.Context(0)
    st = torch.cuda.Stream(dev)
    sh = st.cuda_stream
    g0 = torch.Generator(device=dev)
    g0.manual_seed(SEED)
    EV = torch.rand(16, dtype=torch.float64, device=dev, generator=g0)
    wgt = torch.ones(n, dtype=torch.int32, device=dev)
    sums = torch.zeros(N, dtype=torch.int64, device=dev)
    nodes = []
    t0 = time.time()
    for q in range(N):
        gj = torch.Generator(device=dev)
        gj.manual_seed(SEED + 1 + q)
        x1 = torch.rand(n * 16, dtype=torch.float64, device=dev, generator=gj)
        x1.view(-1, 16)[0::4] *= 1e-12
        x2 = torch.rand(n * 16, dtype=torch.float64, device=dev, generator=gj)
        nodes.append(dict(x1=x1, x2=x2, x3=torch.empty(n * 16, dtype=torch.float64, device=dev),
                          left=torch.rand(64, dtype=torch.float64, device=dev, generator=gj),
                          right=torch.rand(64, dtype=torch.float64, device=dev, generator=gj),
                          scaler=torch.empty(n, dtype=torch.uint8, device=dev),
                          scaler_sum=sums[q:q + 1]))
        if q % 128 == 127:
            print(f"allocated {q + 1} nodes ({time.time() - t0:.0f} s)", flush=True)
    torch.cuda.synchronize()
    G = N // 32
    A = [ctx.bind_plf_batch_dev(nodes[32 * g:32 * g + 32], EV, n, wgt) for g in range(G)]
    B = [ctx.bind_plf_batch_dev(nodes[g::G], EV, n, wgt) for g in range(G)]
    torch.cuda.synchronize()
    res = {}
    for name, sched in (("A consecutive", A), ("B interleaved", B)):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(G + 1)]
        per = [[] for _ in range(G)]
        tot = []
        for r in range(R):
            torch.cuda.synchronize()
            ev[0].record(st)
            for g in range(G):
                sched[g](sh)
                ev[g + 1].record(st)
            torch.cuda.synchronize()
            for g in range(G):
                per[g].append(ev[g].elapsed_time(ev[g + 1]) * 1e3)
            tot.append(ev[0].elapsed_time(ev[G]))
        res[name] = tot
        print(f"== {name}: ms per 512 nodes {[round(t, 2) for t in tot]}; per launch (us, median):")
        print("   " + " ".join(f"{sorted(v)[len(v) // 2]:.0f}" for v in per), flush=True)
    bps = 385 * n * N
    for name, tot in res.items():
        m = sorted(tot)[len(tot) // 2]
        print(f"{name}: {m:.2f} ms = {bps / (m * 1e-3) / 1e9:.0f} GB/s = {bps / (m * 1e-3) / 8e12:.3f} of 8 TB/s")
    s = sums.clone()
    for g in range(G):
        B[g](sh)
    torch.cuda.synchronize()
    print("scaler sums equal under both schedules:", bool(torch.equal(s, sums)))
    ctx.close()


if __name__ == "__main__":
    main()
