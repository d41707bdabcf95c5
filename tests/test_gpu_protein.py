"""GPU tests of the S=20 (protein) kernel, BASELINE configs[4].  The reference
is DNA-only: parity is against the oracle's generic restatement of
the same loop (plfo_plf_gen_*), which reproduces the pinned DNA plf()
bit-for-bit at S=4.  EXACT mode: bit-identical; FMA mode: within 1e-12
relative (one rounding per fused term), identical scaler decisions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S, CAT = 20, 4
V = S * CAT
FMA_RTOL = 1e-12


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gen(n, dtype, seed):
    rng = np.random.default_rng(seed)
    x1 = rng.random(V * n)
    x1.reshape(n, V)[0::4] *= 1e-14          # every 4th site underflows (all 80 values)
    x2 = rng.random(V * n)
    left = rng.random(CAT * S * S)
    right = rng.random(CAT * S * S)
    EV = rng.random(S * S) - 0.25          # signed: some cancellation in the back-transform
    w = rng.integers(0, 4, n).astype(np.int32)
    return [a.astype(dtype) for a in (x1, x2, EV, left, right)] + [w]


def run(ctx, x1, x2, EV, left, right, w, n, fma):
    import torch

    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    x3 = torch.empty(V * n, dtype=t[0].dtype, device="cuda")
    sc = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, t[5], sc, s, n=n, fma=fma)
    torch.cuda.synchronize()
    return x3.cpu().numpy(), sc.cpu().numpy()[:n], int(s.item())


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 257, 3001])
def test_protein_exact_matches_oracle(ctx, oracle, dtype, n):
    x1, x2, EV, left, right, w = gen(max(n, 1), dtype, n)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=False)
    if n == 0:
        assert s == 0
        return
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc
    assert esc.sum() > 0 or n < 4


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [1, 17, 64, 100, 4097])
def test_protein_fma_mode(ctx, oracle, dtype, n):
    """FMA mode (f64: matrix cores, v_mfma_f64_16x16x4 = k-ordered fma chain;
    f32: fused VALU) is bit-identical to the oracle's fma() restatement and
    within 1e-12 (f64) of the unfused loop."""
    x1, x2, EV, left, right, w = gen(n, dtype, 5 + n)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=True)
    f3, fsc, finc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    assert np.array_equal(bits(x3), bits(f3))
    assert np.array_equal(sc, fsc) and s == finc
    if dtype == np.float64:
        e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
        assert np.array_equal(sc, esc) and s == einc
        scale = np.abs(e3).reshape(n, V).max(axis=1, keepdims=True)   # cancellation-aware bound
        err = np.abs(x3 - e3).reshape(n, V) / scale
        assert err.max() <= FMA_RTOL


def test_protein_full_size_256k(ctx, oracle):
    """BASELINE configs[4]: 2^18 sites, f64, bit-exact (EXACT mode), lnL."""
    import torch

    n = 1 << 18
    x1, x2, EV, left, right, w = gen(n, np.float64, 2025)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=False)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc
    freq = np.full(S, 1.0 / S)
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    xs = dev(np.abs(x3))
    ctx.root_lnl(xs, n, out, freq=dev(freq), wgt=dev(w), states=S)
    torch.cuda.synchronize()
    exp = oracle.root_lnl(S, CAT, np.abs(x3), n, freq=freq, wgt=w)
    assert abs(float(out.item()) - exp) <= 1e-12 * abs(exp)
