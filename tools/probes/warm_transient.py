"""warm_transient.py -- probe (not product code): where does the protein
kernel's cold-start transient come from?

Round 2 saw the first ~120 back-to-back launches of the protein f64 FMA kernel
in a fresh process run 96-103 us against a steady 91.5 us, with the shader
clock flat (profiles/r02_probe_clock_drift.log).  That run launched protein
FIRST, so "the DNA kernel shows no drift" was confounded with order.  This
probe separates the candidates, all through the product library (libplfx):

  A  fresh process, DNA f64 node 2^20 first      -> GPU-wide warm-up?
  B  protein right after A                        -> protein-specific?
  C  protein again after 3 s idle                 -> idle/power-state return?
  D  protein on freshly allocated buffers         -> first-touch / TLB?
  E  DNA after 3 s idle

Per launch: HIP-event duration on the launch stream.  Beside it, a thread
samples amdsmi's GPU metrics table (gfx/mem/fabric/soc clocks, socket power,
UMC activity) every ~1 ms; each sample is put on the launch timeline by the
host clock.

  python tools/probes/warm_transient.py [launches=300] > gpurun_out/warm.log
"""
from __future__ import annotations

import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "amd-versal-phylogenetic-likelihood-function_amd"))

import torch  # noqa: E402

import plfx  # noqa: E402

KEYS = ("current_gfxclk", "current_uclk", "current_fclk", "current_socclk", "average_gfxclk_frequency",
        "average_uclk_frequency", "average_fclk_frequency", "current_socket_power",
        "average_socket_power", "average_umc_activity", "average_gfx_activity",
        "temperature_hotspot", "temperature_mem", "firmware_timestamp")


class Sampler(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.samples, self.stop, self.err = [], threading.Event(), None
        self.h = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            self.amdsmi, self.h = amdsmi, hs[0] if hs else None
        except Exception as e:  # noqa: BLE001 -- probe: report and carry on
            self.err = repr(e)

    def run(self):
        if self.h is None:
            return
        while not self.stop.is_set():
            t = time.perf_counter()
            try:
                m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
            except Exception as e:  # noqa: BLE001
                self.err = repr(e)
                return
            self.samples.append((t, {k: m.get(k) for k in KEYS if k in m}))
            time.sleep(0.0005)


def _scalar(v):
    if isinstance(v, (list, tuple)):
        v = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF)]
        return max(v) if v else None
    return v if isinstance(v, (int, float)) else None


def run_pass(name, launch, N, stream, sampler):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
    torch.cuda.synchronize()
    n0 = len(sampler.samples)
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(N):
        launch(i)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    d = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(N)]
    smp = sampler.samples[n0:]
    print(f"== {name}: {N} launches, {sum(d)/1e3:.1f} ms GPU, host {1e3*(t1-t0):.1f} ms; "
          f"{len(smp)} metric samples")
    # launch k starts ~ at t0 + sum(d[:k]) (launches queue faster than they run)
    starts, acc = [], 0.0
    for x in d:
        starts.append(t0 + acc * 1e-6)
        acc += x
    W = 20
    for w in range(0, N, W):
        seg = sorted(d[w:w + W])
        ta, tb = starts[w], starts[min(w + W, N - 1)] + d[min(w + W, N - 1)] * 1e-6
        ms = [s for (t, s) in smp if ta <= t < tb]
        desc = ""
        if ms:
            def avg(k):
                v = [_scalar(s.get(k)) for s in ms]
                v = [x for x in v if x is not None]
                return sum(v) / len(v) if v else None
            parts = []
            for k, lab in (("current_gfxclk", "gfx"), ("current_uclk", "uclk"), ("current_fclk", "fclk"),
                           ("current_socclk", "soc"), ("current_socket_power", "W"),
                           ("average_umc_activity", "umc%"), ("temperature_hotspot", "Thot"),
                           ("temperature_mem", "Tmem")):
                v = avg(k)
                if v is not None:
                    parts.append(f"{lab} {v:.0f}")
            desc = " | " + " ".join(parts) + f" ({len(ms)} smp)"
        print(f"  [{w:4d}..{min(w+W, N):4d}) median {seg[len(seg)//2]:7.1f} us  min {seg[0]:7.1f}{desc}")
    return d


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda", 0)
    ctx = plfx.Context(0)
    st = torch.cuda.Stream(dev)
    sh = st.cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    sampler = Sampler()
    print("amdsmi:", "ok" if sampler.h is not None else f"unavailable {sampler.err}")
    if sampler.h is not None:
        m = sampler.amdsmi.amdsmi_get_gpu_metrics_info(sampler.h)
        print("metrics keys with values:", {k: m[k] for k in KEYS if k in m})
    sampler.start()

    def dna_sets(R=4):
        n = 1 << 20
        S = []
        for _ in range(R):
            x1 = torch.rand(16 * n, dtype=torch.float64, device=dev, generator=g)
            x2 = torch.rand(16 * n, dtype=torch.float64, device=dev, generator=g)
            S.append(dict(x1=x1, x2=x2, x3=torch.empty_like(x1),
                          wgt=torch.ones(n, dtype=torch.int32, device=dev),
                          sc=torch.empty(n, dtype=torch.uint8, device=dev),
                          s=torch.zeros(1, dtype=torch.int64, device=dev)))
        return S

    def prot_sets(R=4):
        n = 1 << 18
        S = []
        for _ in range(R):
            x1 = torch.rand(80 * n, dtype=torch.float64, device=dev, generator=g)
            x1.view(-1, 80)[0::4] *= 1e-14
            x2 = torch.rand(80 * n, dtype=torch.float64, device=dev, generator=g)
            S.append(dict(x1=x1, x2=x2, x3=torch.empty_like(x1),
                          wgt=torch.ones(n, dtype=torch.int32, device=dev),
                          sc=torch.empty(n, dtype=torch.uint8, device=dev),
                          s=torch.zeros(1, dtype=torch.int64, device=dev)))
        return S

    EV4 = torch.rand(16, dtype=torch.float64, device=dev, generator=g) - 0.25
    L4 = torch.rand(64, dtype=torch.float64, device=dev, generator=g)
    R4 = torch.rand(64, dtype=torch.float64, device=dev, generator=g)
    EV20 = torch.rand(400, dtype=torch.float64, device=dev, generator=g) - 0.25
    L20 = torch.rand(1600, dtype=torch.float64, device=dev, generator=g)
    R20 = torch.rand(1600, dtype=torch.float64, device=dev, generator=g)
    D = dna_sets()
    P = prot_sets()
    torch.cuda.synchronize()
    time.sleep(3.0)   # settle: start every pass from the same idle state

    def dna(S):
        return lambda i: ctx.plf_dev(S[i % 4]["x1"], S[i % 4]["x2"], S[i % 4]["x3"], EV4, L4, R4,
                                     S[i % 4]["wgt"], S[i % 4]["sc"], S[i % 4]["s"], stream=sh)

    def prot(S):
        return lambda i: ctx.plf_dev_gen(S[i % 4]["x1"], S[i % 4]["x2"], S[i % 4]["x3"], EV20, L20,
                                         R20, 20, S[i % 4]["wgt"], S[i % 4]["sc"], S[i % 4]["s"],
                                         fma=True, stream=sh)

    run_pass("A dna f64 2^20 (first kernel of the process, after 3 s idle)", dna(D), N, st, sampler)
    run_pass("B protein f64 FMA 2^18 (right after A)", prot(P), N, st, sampler)
    time.sleep(3.0)
    run_pass("C protein again after 3 s idle", prot(P), N, st, sampler)
    P2 = prot_sets()
    torch.cuda.synchronize()
    run_pass("D protein on freshly allocated buffers (no idle)", prot(P2), N, st, sampler)
    del P2
    time.sleep(3.0)
    run_pass("E dna after 3 s idle", dna(D), N, st, sampler)
    run_pass("F protein right after E", prot(P), N, st, sampler)
    time.sleep(0.3)
    run_pass("G protein after 0.3 s idle", prot(P), N, st, sampler)
    sampler.stop.set()
    sampler.join(timeout=2)
    if sampler.err:
        print("sampler error:", sampler.err)
    ctx.close()


if __name__ == "__main__":
    main()
