#!/usr/bin/env python3
"""Probe (not product code): does the dependent-launch gap of the headline
node line (69.2 us event time per step against 67.5 us of kernel)
close when consecutive steps -- independent nodes on different buffer sets --
are issued on more than one stream, so one node's last blocks overlap the next
node's first?  bench.py's node workload (f64, 2^20 sites, 4 buffer sets),
steps captured in one HIP graph as the bench does:
  s1      every step on the launch stream (the bench today)
  s2, s4  step i on stream i % S: fork from the launch stream at the start of
          the capture, join at its end (buffer set i % 4 stays on one stream)
  g2      two single-stream graphs, even steps on the launch stream and odd
          steps on a second stream (which first waits for the launch stream)
  e1, e2  S = 1 / 2 without a graph (host launches)
  e2n     e2 without the closing join on the device: an end event on each
          stream (device time = the later one), the host waits for the device
  e2f     e2n with the first step launched before the second stream's wait
          (on the region's start event, no new event)
  g2f     g2 the same way: the even-step graph launched first, the odd-step
          graph's stream waits on the start event, no join on the device
  h2f     g2f with step 0 launched directly and the even-step graph from step 2
  g2c     g2f through the HIP API directly (ctypes hipGraphLaunch /
          hipStreamWaitEvent / hipEventRecord: no torch replay() around it)
  gc3,gc4 g2c over 3 / 4 lanes (--sets must be a multiple of the lanes)
  g2h     g2c with the context told two calls are in flight
          (plfx_ctx_set_streams 2: half grids; the bench's form)
  g2e     g2h with the region's first and last steps at the full grid (they
          run partly alone)
  g2n     g2h without lane 1's wait on the start event: each lane records its
          own start event; device time from the earlier start to the later end
--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is touched.
Each variant's event time per step around one replay and its host wall from
before the launch to after the synchronize (what bench.py's `value` divides
by), variants alternating, median of the reps; after every replay each buffer set's x3 / scaler bytes /
scaler sum must equal the single-stream result bit for bit.

  python3 tools/probes/node_overlap.py [--steps 20,200] [--reps 11] [--dtype f64] [--only s1,e2]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="20,200")
    ap.add_argument("--reps", type=int, default=11)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--only", default="", help="comma-separated variants (default: all)")
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--sets", type=int, default=4, help="buffer sets")
    o = ap.parse_args()
    if o.spin:
        import ctypes as C
        rc = C.CDLL("libamdhip64.so").hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
        print(f"hipSetDeviceFlags(spin) -> {rc}", flush=True)
    dev = torch.device("cuda", 0)
    esz = 8 if o.dtype == "f64" else 4
    tdt = torch.float64 if esz == 8 else torch.float32
    a = bench.parse(["--steps", "20", "--warmup", "5", "--dtype", o.dtype, "--buffer-sets", str(o.sets)])
    ctx = plfx.Context(0, lazy_tables=True)
    wl = bench.NodeWorkload(ctx, a, dev, None, tdt, esz)
    main_s = torch.cuda.Stream(dev)
    side = [torch.cuda.Stream(dev) for _ in range(3)]
    for st_ in [main_s] + side:  # every stream's workspace exists before any capture
        for i in range(4):
            wl.step(i, st_.cuda_stream)
        torch.cuda.synchronize()
    want = [(b["x3"].clone(), b["sc"].clone(), b["s"].clone()) for b in wl.sets]

    def issue(K, S, join=True):
        streams = [main_s] + side[:S - 1]
        for s in streams[1:]:
            s.wait_stream(main_s)
        for i in range(K):
            wl.step(i, streams[i % S].cuda_stream)
        if join:
            for s in streams[1:]:
                main_s.wait_stream(s)

    def graph(K, S):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            issue(K, S)
        torch.cuda.synchronize()
        return g

    def half(K, parity, s, skip=0, L=2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(parity + skip, K, L):
                wl.step(i, s.cuda_stream)
        torch.cuda.synchronize()
        return g

    def half_sched(K, parity, s, full=()):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(parity, K, 2):
                ctx.set_streams(1 if i in full else 2)
                wl.step(i, s.cuda_stream)
        ctx.set_streams(1)
        torch.cuda.synchronize()
        return g

    def run_g2(pair):
        ga, gb = pair
        side[0].wait_stream(main_s)
        with torch.cuda.stream(main_s):
            ga.replay()
        with torch.cuda.stream(side[0]):
            gb.replay()
        main_s.wait_stream(side[0])

    def same():
        for b, (x3, sc, s) in zip(wl.sets, want):
            if not (torch.equal(b["x3"].view(torch.int64 if esz == 8 else torch.int32),
                                x3.view(torch.int64 if esz == 8 else torch.int32))
                    and torch.equal(b["sc"], sc) and torch.equal(b["s"], s)):
                return False
        return True

    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    bytes_step = bench.bytes_per_site(esz) * wl.n
    for K in [int(x) for x in o.steps.split(",")]:
        gs = {f"s{S}": graph(K, S) for S in (1, 2, 4)}
        gs["g2"] = (half(K, 0, main_s), half(K, 1, side[0]))
        gs["g2f"] = gs["g2"]
        gs["h2f"] = (half(K, 0, main_s, skip=2), gs["g2"][1])
        gs["g2c"] = gs["g2"]
        if "g2h" in o.only.split(","):
            gs["g2h"] = (half_sched(K, 0, main_s), half_sched(K, 1, side[0]))
        if "g2n" in o.only.split(","):
            gs["g2n"] = (half_sched(K, 0, main_s), half_sched(K, 1, side[0]))
        if "g2e" in o.only.split(","):
            gs["g2e"] = (half_sched(K, 0, main_s, (0, K - 1)), half_sched(K, 1, side[0], (0, K - 1)))
        for L in (3, 4):
            if f"gc{L}" in o.only.split(",") and o.sets % L == 0:
                gs[f"gc{L}"] = tuple(half(K, l, ([main_s] + side)[l], L=L) for l in range(L))
        res = {k: [] for k in list(gs) + ["e1", "e2", "e2n", "e2f"] if not o.only or k in o.only.split(",")}
        wall = {k: [] for k in res}
        ok = True
        for _ in range(o.reps):
            for k in res:
                for i in range(4):  # a short warm-up on the launch stream
                    wl.step(i, main_s.cuda_stream)
                with torch.cuda.stream(main_s):  # then outputs cleared: the replay must write them
                    for b in wl.sets:
                        b["x3"].zero_()
                        b["sc"].zero_()
                        b["s"].zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e1b = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                if k == "g2n":
                    e0b = torch.cuda.Event(enable_timing=True)
                    ends = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    lanes = [main_s, side[0]]
                    for e, st_ in ((e0, main_s), (e0b, side[0])):
                        e.record(st_)
                    for e, st_ in zip(ends, lanes):
                        e.record(st_)
                    torch.cuda.synchronize()
                    ex = [C.c_void_p(int(g.raw_cuda_graph_exec())) for g in gs[k]]
                    hl = [C.c_void_p(st_.cuda_stream) for st_ in lanes]
                    starts = [C.c_void_p(e0.cuda_event), C.c_void_p(e0b.cuda_event)]
                    t0 = time.perf_counter()
                    for h, x, es in zip(hl, ex, starts):
                        hip.hipEventRecord(es, h)
                        hip.hipGraphLaunch(x, h)
                    for h, e in zip(hl, ends):
                        hip.hipEventRecord(C.c_void_p(e.cuda_event), h)
                    hip.hipDeviceSynchronize()
                    wall[k].append((time.perf_counter() - t0) * 1e6 / K)
                    first = e0 if e0.elapsed_time(e0b) >= 0 else e0b
                    res[k].append(max(first.elapsed_time(e) for e in ends) * 1e3 / K)
                    ok = ok and same()
                    continue
                if k in ("g2c", "gc3", "gc4", "g2h", "g2e"):
                    lanes = [main_s] + side[:len(gs[k]) - 1]
                    ends = [torch.cuda.Event(enable_timing=True) for _ in lanes]
                    e0.record(main_s)  # creates the HIP events
                    for e, st_ in zip(ends, lanes):
                        e.record(st_)
                    torch.cuda.synchronize()
                    ex = [C.c_void_p(int(g.raw_cuda_graph_exec())) for g in gs[k]]
                    hl = [C.c_void_p(st_.cuda_stream) for st_ in lanes]
                    he0 = C.c_void_p(e0.cuda_event)
                    t0 = time.perf_counter()
                    hip.hipEventRecord(he0, hl[0])
                    for j, (h, x) in enumerate(zip(hl, ex)):
                        if j:
                            hip.hipStreamWaitEvent(h, he0, 0)
                        hip.hipGraphLaunch(x, h)
                    for h, e in zip(hl, ends):
                        hip.hipEventRecord(C.c_void_p(e.cuda_event), h)
                    hip.hipDeviceSynchronize()
                    wall[k].append((time.perf_counter() - t0) * 1e6 / K)
                    res[k].append(max(e0.elapsed_time(e) for e in ends) * 1e3 / K)
                    ok = ok and same()
                    continue
                t0 = time.perf_counter()
                e0.record(main_s)
                if k == "e2n":
                    issue(K, 2, join=False)
                    e1b.record(side[0])
                elif k == "e2f":
                    wl.step(0, main_s.cuda_stream)
                    side[0].wait_event(e0)
                    for i in range(1, K):
                        wl.step(i, (side[0] if i % 2 else main_s).cuda_stream)
                    e1b.record(side[0])
                elif k in ("g2f", "h2f"):
                    if k == "h2f":
                        wl.step(0, main_s.cuda_stream)
                    with torch.cuda.stream(main_s):
                        gs[k][0].replay()
                    side[0].wait_event(e0)
                    with torch.cuda.stream(side[0]):
                        gs[k][1].replay()
                    e1b.record(side[0])
                elif k in ("e1", "e2"):
                    issue(K, int(k[1]))
                elif k == "g2":
                    run_g2(gs[k])
                else:
                    with torch.cuda.stream(main_s):
                        gs[k].replay()
                e1.record(main_s)
                torch.cuda.synchronize()
                wall[k].append((time.perf_counter() - t0) * 1e6 / K)
                d = e0.elapsed_time(e1)
                if k in ("e2n", "e2f", "g2f", "h2f"):
                    d = max(d, e0.elapsed_time(e1b))
                res[k].append(d * 1e3 / K)
                ok = ok and same()
        for k, v in res.items():
            m = st.median(v)
            w = st.median(wall[k])
            print(f"{o.dtype} K={K:4d} {k:3s} events {m:7.2f} us/step (min {min(v):7.2f}, max {max(v):7.2f}) "
                  f"frac {bytes_step / (m * 1e-6) / 8e12:.4f}; wall {w:7.2f} us/step "
                  f"frac {bytes_step / (w * 1e-6) / 8e12:.4f}", flush=True)
        print(f"{o.dtype} K={K} every replay bit-identical to the single-stream outputs: {ok}", flush=True)
        del gs
    ctx.close()


if __name__ == "__main__":
    main()
