# A/B (tuning only, round 3; the switch it flips was removed after the run,
# profiles/r03_host_split_uploads.log): host-array entry with both uploads on one stream (0) vs
# the right child's upload on its own stream (1), alternating, same process.
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, 'amd-versal-phylogenetic-likelihood-function_amd')
import plfx
ctx = plfx.Context(0)
res = {}
for pinned in (False, True):
    for dtype in (np.float64, np.float32):
        n = 1 << 20
        rng = np.random.default_rng(1)
        tdt = torch.float64 if dtype == np.float64 else torch.float32
        def buf(v):
            if not pinned:
                return np.ascontiguousarray(v)
            t = torch.empty(v.size, dtype=tdt, pin_memory=True); a = t.numpy(); a[:] = v; return a
        x1, x2 = buf(rng.random(16 * n).astype(dtype)), buf(rng.random(16 * n).astype(dtype))
        x3 = buf(np.zeros(16 * n, dtype))
        EV, L, R = rng.random(16).astype(dtype), rng.random(64).astype(dtype), rng.random(64).astype(dtype)
        w = np.ones(n, np.int32)
        outs = {}
        for rnd in range(3):
            for split in (0, 1):
                os.environ["PLFX_TMP_HOST_SPLIT"] = str(split)
                ctx.plf(x1, x2, x3, EV, n, L, R, w)
                reps, t0 = 0, time.perf_counter()
                while time.perf_counter() - t0 < 1.0:
                    ctx.plf(x1, x2, x3, EV, n, L, R, w); reps += 1
                el = time.perf_counter() - t0
                res.setdefault((pinned, np.dtype(dtype).name, split), []).append(reps * n / el)
                outs[split] = x3.copy()
        assert np.array_equal(outs[0], outs[1])
for k, v in res.items():
    print(f"{'pinned  ' if k[0] else 'pageable'} {k[1]} split={k[2]}: median {sorted(v)[1]:.3e} sites/s  all {[f'{x:.3e}' for x in v]}")
