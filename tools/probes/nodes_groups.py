"""nodes_groups.py -- probe (not product code): why do the 16 batched 32-node
launches of nodes512 (BASELINE configs[3]) at N = 1 split into ~2.11 ms and
~2.39 ms groups (profiles/r02_nodes512_launch_groups.log)?

Same allocation as bench.py's NodesWorkload (one torch tensor per CLV, 512
nodes x 3 CLVs x 2^20 f64 sites = 201 GB).  Then:

  1. each 32-node launch group, timed over several rounds   -> slow / fast groups
  2. every node of two slow and two fast groups ALONE (count-1 batch) -> is a
     slow group made of slow nodes (a property of its allocations), or only
     slow together (an interaction of its 96 streams)?
  3. mixed groups: half the nodes of a slow group + half of a fast one
  5. the same nodes in launches of 8 and 16
  6. node j of a group entered at site j*delta: the concurrent streams'
     relative alignment shifted by j*delta*128 B
  4. per node, the buffers' virtual addresses (mod 2 MiB / 1 GiB and the gap
     to the previous allocation), to correlate with the timings

  python tools/probes/nodes_groups.py [nodes=512] [sites=1048576] > gpurun_out/nodes_groups.log
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
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
        x3 = torch.empty(n * 16, dtype=torch.float64, device=dev)
        nodes.append(dict(x1=x1, x2=x2, x3=x3,
                          left=torch.rand(64, dtype=torch.float64, device=dev, generator=gj),
                          right=torch.rand(64, dtype=torch.float64, device=dev, generator=gj),
                          scaler=torch.empty(n, dtype=torch.uint8, device=dev),
                          scaler_sum=sums[q:q + 1]))
        if q % 64 == 63:
            print(f"allocated {q + 1} nodes ({time.time() - t0:.0f} s)", flush=True)
    torch.cuda.synchronize()

    def timed(fn, reps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        torch.cuda.synchronize()
        e[0].record(st)
        for r in range(reps):
            fn()
            e[r + 1].record(st)
        torch.cuda.synchronize()
        return [e[r].elapsed_time(e[r + 1]) * 1e3 for r in range(reps)]

    G = (N + 31) // 32
    groups = [ctx.bind_plf_batch_dev(nodes[i:i + 32], EV, n, wgt) for i in range(0, N, 32)]
    for _ in range(3):  # past the clock transient
        for gr in groups:
            gr(sh)
    torch.cuda.synchronize()
    print("== 1. launch groups (us per 32-node launch), 4 rounds", flush=True)
    gt = [[] for _ in range(G)]
    for r in range(4):
        for k in range(G):
            gt[k] += timed(lambda: groups[k](sh), 1)
    med = [sorted(v)[len(v) // 2] for v in gt]
    for k in range(G):
        print(f"  group {k:2d}: " + " ".join(f"{x:7.0f}" for x in gt[k]) + f"   median {med[k]:7.0f}")
    order = sorted(range(G), key=lambda k: med[k])
    fast, slow = order[:2], order[-2:]
    print(f"fastest groups {fast}, slowest {slow}", flush=True)

    print("== 2. nodes alone (us per single-node launch, median of 3)", flush=True)
    for k in fast + slow:
        row = []
        for q in range(32 * k, min(32 * k + 32, N)):
            one = ctx.bind_plf_batch_dev(nodes[q:q + 1], EV, n, wgt)
            v = sorted(timed(lambda: one(sh), 3))
            row.append(v[1])
        print(f"  group {k:2d} ({'fast' if k in fast else 'slow'}): mean {sum(row)/len(row):6.1f} "
              f"min {min(row):6.1f} max {max(row):6.1f} | " + " ".join(f"{x:.0f}" for x in row), flush=True)

    print("== 3. mixed groups (16 nodes of a slow group + 16 of a fast one)", flush=True)
    for a, b in ((slow[0], fast[0]), (slow[1], fast[1])):
        mix = nodes[32 * a:32 * a + 16] + nodes[32 * b:32 * b + 16]
        lm = ctx.bind_plf_batch_dev(mix, EV, n, wgt)
        v = sorted(timed(lambda: lm(sh), 4))
        mix2 = nodes[32 * a + 16:32 * a + 32] + nodes[32 * b + 16:32 * b + 32]
        lm2 = ctx.bind_plf_batch_dev(mix2, EV, n, wgt)
        v2 = sorted(timed(lambda: lm2(sh), 4))
        print(f"  slow {a} first half + fast {b} first half: {v[1]:.0f} us; second halves: {v2[1]:.0f} us")
        # the slow group's nodes in another order (reversed): same addresses, other blockIdx.y
        rev = list(reversed(nodes[32 * a:32 * a + 32]))
        lr = ctx.bind_plf_batch_dev(rev, EV, n, wgt)
        v3 = sorted(timed(lambda: lr(sh), 4))
        print(f"  slow {a} reversed node order: {v3[1]:.0f} us", flush=True)

    print("== 5. smaller batches of the same nodes (us per 32 nodes)", flush=True)
    for k in (slow + fast):
        for cnt in (8, 16):
            ls = [ctx.bind_plf_batch_dev(nodes[32 * k + i:32 * k + i + cnt], EV, n, wgt)
                  for i in range(0, 32, cnt)]
            v = sorted(timed(lambda: [f(sh) for f in ls], 4))
            print(f"  group {k:2d} ({'fast' if k in fast else 'slow'}) in launches of {cnt}: {v[1]:.0f} us", flush=True)

    print("== 6. node j's buffers entered at site j*delta (n' = n - 31*delta): does shifting the "
          "concurrent streams' relative alignment change a group's time?", flush=True)
    for k in (slow + fast):
        row = []
        for delta in (0, 1, 8, 64, 512, 4096, 16384):
            m = n - 31 * delta
            sub = []
            for j, q in enumerate(range(32 * k, 32 * k + 32)):
                o = j * delta
                nd = dict(nodes[q])
                for key in ("x1", "x2", "x3"):
                    nd[key] = nodes[q][key][16 * o:16 * (o + m)]
                nd["scaler"] = nodes[q]["scaler"][o:o + m]
                sub.append(nd)
            f = ctx.bind_plf_batch_dev(sub, EV, m, wgt)
            v = sorted(timed(lambda: f(sh), 4))
            row.append(f"d={delta}: {v[1] * n / m:.0f}")
        print(f"  group {k:2d} ({'fast' if k in fast else 'slow'}), us scaled to n sites: " + "  ".join(row),
              flush=True)

    print("== 4. buffer addresses per group (x1/x2/x3 data_ptr mod 2 MiB, GiB of first x1)")
    for k in range(G):
        mods = set()
        for q in range(32 * k, min(32 * k + 32, N)):
            for key in ("x1", "x2", "x3"):
                mods.add(nodes[q][key].data_ptr() % (2 << 20))
        p0 = nodes[32 * k]["x1"].data_ptr()
        print(f"  group {k:2d} ({med[k]:6.0f} us): first x1 at {p0 / 2**30:9.3f} GiB, "
              f"offsets mod 2 MiB {sorted(mods)[:4]}{'...' if len(mods) > 4 else ''}")
    ctx.close()


if __name__ == "__main__":
    main()
