# Host-array entry (plfx_plf_f32/f64) rate, PCIe-inclusive (tuning only): pageable
# numpy buffers as plf()'s callers pass them, and page-locked buffers (torch
# pin_memory) with which the chunked H2D / D2H pipeline can overlap directions.
import sys
import time

import numpy as np
import torch

sys.path.insert(0, 'amd-versal-phylogenetic-likelihood-function_amd')
import plfx  # noqa: E402

ctx = plfx.Context(0)
for pinned in (False, True):
    for dtype in (np.float64, np.float32):
        for n in (1 << 18, 1 << 20, 1 << 22):
            rng = np.random.default_rng(1)
            tdt = torch.float64 if dtype == np.float64 else torch.float32

            def buf(v):
                if not pinned:
                    return np.ascontiguousarray(v)
                t = torch.empty(v.size, dtype=tdt, pin_memory=True)
                a = t.numpy()
                a[:] = v
                return a
            x1, x2 = buf(rng.random(16 * n).astype(dtype)), buf(rng.random(16 * n).astype(dtype))
            x3 = buf(np.zeros(16 * n, dtype))
            EV, L, R = rng.random(16).astype(dtype), rng.random(64).astype(dtype), rng.random(64).astype(dtype)
            w = np.ones(n, np.int32)
            ctx.plf(x1, x2, x3, EV, n, L, R, w)
            reps, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < 1.5:
                ctx.plf(x1, x2, x3, EV, n, L, R, w)
                reps += 1
            el = time.perf_counter() - t0
            gbs = reps * n * 48 * np.dtype(dtype).itemsize / el / 1e9
            print(f"{'pinned  ' if pinned else 'pageable'} {np.dtype(dtype).name} n={n}: "
                  f"{reps * n / el:.3e} sites/s ({gbs:.1f} GB/s both directions)")
