#!/usr/bin/env python3
"""Probe (not product code): host wall of the FIRST replay of an instantiated
HIP graph vs later replays, for bench.py's node workload (20 steps of the
headline kernel captured in one graph, as the driver's `--steps 20` runs it),
with and without hipGraphUpload before the first replay.  The driver's timed
region is one replay; a first-replay cost lands in `value`.

  python3 tools/probes/graph_first_replay.py
"""
import ctypes as C
import statistics as st
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import plfx  # noqa: E402


def main():
    a = bench.parse(["--steps", "20", "--warmup", "5", "--no-nodes512"])
    dev = torch.device("cuda", 0)
    ctx = plfx.Context(0, lazy_tables=True)
    wl = bench.NodeWorkload(ctx, a, dev, None, torch.float64, 8)
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream
    hip = C.CDLL("libamdhip64.so")
    for i in range(8):
        wl.step(i, sh)
    torch.cuda.synchronize()

    def make(upload):
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=stream):
            for i in range(a.steps):
                wl.step(i, sh)
        g.instantiate()
        if upload:
            rc = hip.hipGraphUpload(C.c_void_p(int(g.raw_cuda_graph_exec())), C.c_void_p(sh))
            assert rc == 0, rc
        torch.cuda.synchronize()
        return g

    def replay_us(g):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    rows = {"plain": [], "upload": []}
    for rep in range(5):
        for mode in ("plain", "upload"):
            g = make(mode == "upload")
            # a few warm-up steps outside the graph, as bench.py runs them
            for i in range(a.warmup):
                wl.step(i, sh)
            torch.cuda.synchronize()
            first = replay_us(g)
            later = [replay_us(g) for _ in range(3)]
            rows[mode].append((first, st.median(later)))
            del g
    for mode, r in rows.items():
        f = [x[0] for x in r]
        lt = [x[1] for x in r]
        print(f"{mode:7s} first replay {st.median(f):8.1f} us (min {min(f):.1f}), later replays "
              f"{st.median(lt):8.1f} us -> first-replay excess {st.median(f) - st.median(lt):6.1f} us "
              f"over {a.steps} steps")
    ctx.close()


if __name__ == "__main__":
    main()
