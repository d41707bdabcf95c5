"""Probe (not product code): how much of bench.py's wall-clock region is the
host waking up after the GPU finished.  A graph of K headline node launches
(2^20 f64 sites, 4 rotating buffer sets) is replayed with the region ended by
(a) torch.cuda.synchronize() alone (a blocking wait) and (b) polling the end
event (hipEventQuery) first, alternating; printed: wall - events per region.

    python tools/probes/sync_latency.py [K ...]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402


def main():
    ks = [int(a) for a in sys.argv[1:]] or [20, 200]
    n = 1 << 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ctx = plfx.Context(0)
    EV = torch.rand(16, dtype=torch.float64, device=dev, generator=g)
    L = torch.rand(64, dtype=torch.float64, device=dev, generator=g)
    R = torch.rand(64, dtype=torch.float64, device=dev, generator=g)
    w = torch.ones(n, dtype=torch.int32, device=dev)
    sets, keep = [], []  # the launchers hold raw pointers: keep every tensor alive
    for _ in range(4):
        x1 = torch.rand(16 * n, dtype=torch.float64, device=dev, generator=g)
        x2 = torch.rand(16 * n, dtype=torch.float64, device=dev, generator=g)
        x3 = torch.empty_like(x1)
        s = torch.zeros(1, dtype=torch.int64, device=dev)
        keep += [x1, x2, x3, s]
        sets.append(ctx.bind_plf_dev(x1, x2, x3, EV, L, R, w, None, s))
    stream = torch.cuda.Stream(dev)
    for k in ks:
        for i in range(8):
            sets[i % 4](stream.cuda_stream)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for i in range(k):
                sets[i % 4](stream.cuda_stream)
        torch.cuda.synchronize(dev)
        res = {"blocking": [], "poll": []}
        for rep in range(12):
            for mode in ("blocking", "poll"):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                e0.record(stream)
                with torch.cuda.stream(stream):
                    graph.replay()
                e1.record(stream)
                if mode == "poll":
                    while not e1.query():
                        pass
                torch.cuda.synchronize(dev)
                wall = (time.perf_counter() - t0) * 1e3
                res[mode].append((wall - e0.elapsed_time(e1)) * 1e3)
        for mode, v in res.items():
            v = sorted(v[2:])
            print(f"K={k:4d} {mode:8s}: wall - events = median {v[len(v) // 2]:7.1f} us "
                  f"(min {v[0]:7.1f}, max {v[-1]:7.1f})", flush=True)
    torch.cuda.synchronize(dev)
    ctx.close()
    del keep


if __name__ == "__main__":
    main()
