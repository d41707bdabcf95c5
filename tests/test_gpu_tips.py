"""GPU tests of tip children (plfx.h section 8).

A tip is one uint8 state code per site; the reference has no tip path (its
plf() takes two dense CLVs), so the definition checked here is plf() -- the
pinned oracle -- on the expanded dense CLV (oracle.expand_tips).  Bar: CLVs,
scaler bytes and scaler sums bit-exact, f32 and f64."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kind", ["tip_tip", "tip_inner", "inner_tip"])
@pytest.mark.parametrize("n", [0, 1, 7, 8, 63, 4099, 65537])
def test_single_node_tips(ctx, oracle, dtype, kind, n):
    import torch

    rng = np.random.default_rng(n * 7 + len(kind))
    c1 = oracle.random_tip_codes(rng, n, 0.2)
    c2 = oracle.random_tip_codes(rng, n, 0.2)
    x1 = oracle.expand_tips(c1, dtype) if kind != "inner_tip" else rng.random(16 * n).astype(dtype)
    x2 = oracle.expand_tips(c2, dtype) if kind != "tip_inner" else rng.random(16 * n).astype(dtype)
    if kind != "tip_tip" and n > 10:  # drive part of the sites through the scaler
        (x1 if kind == "inner_tip" else x2)[16 * (n // 3):16 * (n // 2)] *= 1e-40 if dtype == np.float64 else 1e-20
    L = (rng.random(64) * 0.5).astype(dtype)
    R = (rng.random(64) * 0.5).astype(dtype)
    EV = rng.random(16).astype(dtype)
    w = rng.integers(0, 4, n).astype(np.int32)
    e3, esc, einc = oracle.plf(x1, x2, EV, L, R, w, n=n)
    tt = torch.float64 if dtype == np.float64 else torch.float32
    x3 = torch.full((max(16 * n, 16),), float("nan"), dtype=tt, device="cuda")
    sc = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
    ss = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    args = dict(wgt=dev(w) if n else None, scaler=sc, scaler_sum=ss)
    if kind in ("tip_tip", "tip_inner"):
        args["tip1"] = dev(c1) if n else torch.zeros(1, dtype=torch.uint8, device="cuda")
    else:
        args["x1"] = dev(x1) if n else torch.zeros(16, dtype=tt, device="cuda")
    if kind in ("tip_tip", "inner_tip"):
        args["tip2"] = dev(c2) if n else torch.zeros(1, dtype=torch.uint8, device="cuda")
    else:
        args["x2"] = dev(x2) if n else torch.zeros(16, dtype=tt, device="cuda")
    ctx.plf_tips_dev(x3, dev(EV), n, dev(L), dev(R), **args)
    torch.cuda.synchronize()
    assert int(ss.item()) == einc
    if n:
        assert np.array_equal(bits(x3.cpu().numpy()[:16 * n]), bits(e3))
        assert np.array_equal(sc.cpu().numpy()[:n], esc)
    if kind != "tip_tip" and n > 10:
        assert esc.sum() > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kind", ["tip_tip", "tip_inner"])
def test_tip_vector_table(ctx, oracle, dtype, kind):
    """A caller-supplied 16 x 4 tip-vector table (e.g. eigen-coordinate tips,
    plfx_model_tip_vectors): bit-exact vs plf() on x[i][c][s] = tv[code_i][s]."""
    import torch

    n = 5003
    rng = np.random.default_rng(77)
    tv = (rng.random(64) * 2 - 0.5).astype(dtype)
    c1 = oracle.random_tip_codes(rng, n, 0.5)
    c2 = oracle.random_tip_codes(rng, n, 0.5)
    x1 = oracle.expand_tips(c1, dtype, tipvec=tv)
    x2 = oracle.expand_tips(c2, dtype, tipvec=tv) if kind == "tip_tip" else rng.random(16 * n).astype(dtype)
    L, R, EV = (rng.random(64).astype(dtype), rng.random(64).astype(dtype),
                rng.random(16).astype(dtype))
    e3, esc, einc = oracle.plf(x1, x2, EV, L, R)
    x3 = torch.empty(16 * n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device="cuda")
    ss = torch.zeros(1, dtype=torch.int64, device="cuda")
    args = dict(tip1=dev(c1), scaler_sum=ss, tipvec=dev(tv))
    if kind == "tip_tip":
        args["tip2"] = dev(c2)
    else:
        args["x2"] = dev(x2)
    ctx.plf_tips_dev(x3, dev(EV), n, dev(L), dev(R), **args)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(e3))
    assert int(ss.item()) == einc


def test_tip_tip_all_codes_scale(ctx, oracle):
    """Code 0 (no state possible) gives an all-zero site: scaled (0 < 2^-32),
    stays 0; a weight per site reaches the sum."""
    import torch

    n = 4096
    codes = np.arange(n, dtype=np.int64).astype(np.uint8)  # every byte value
    rng = np.random.default_rng(5)
    L, R, EV = rng.random(64), rng.random(64), rng.random(16)
    w = rng.integers(1, 9, n).astype(np.int32)
    e3, esc, einc = oracle.plf(oracle.expand_tips(codes), oracle.expand_tips(codes[::-1].copy()),
                               EV, L, R, w)
    x3 = torch.empty(16 * n, dtype=torch.float64, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    ss = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_tips_dev(x3, dev(EV), n, dev(L), dev(R), tip1=dev(codes), tip2=dev(codes[::-1].copy()),
                     wgt=dev(w), scaler=sc, scaler_sum=ss)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(e3))
    assert np.array_equal(sc.cpu().numpy(), esc)
    assert int(ss.item()) == einc and einc > 0


def _tree_with_tips(oracle, ntips, n, dtype, seed, coded):
    rng = np.random.default_rng(seed)
    ops = oracle.balanced_tree_ops(ntips)
    nslots = ntips + ops.shape[0]
    codes = [oracle.random_tip_codes(rng, n, 0.1) for _ in range(ntips)]
    dense = [rng.random(16 * n).astype(dtype) for _ in range(ntips)]
    pm = (rng.random(ops.shape[0] * 128) * 0.25).astype(dtype)
    EV = (rng.random(16) * 0.25).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_tips(codes[t], dtype) if coded[t] else dense[t].copy() for t in range(ntips)]
    host += [np.zeros(16 * n, dtype) for _ in range(nslots - ntips)]
    return ops, nslots, codes, dense, pm, EV, wgt, host


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("pattern", ["all", "mixed"])
def test_traverse_with_tips(ctx, oracle, dtype, pattern):
    """Balanced 16-taxon tree: all tips coded (level 0 = tip/tip), or a mix
    (tip/tip, tip/inner, inner/tip and inner/inner in one level)."""
    import torch

    n = 2049
    ntips = 16
    coded = [True] * ntips if pattern == "all" else [t % 3 != 1 for t in range(ntips)]
    ops, nslots, codes, dense, pm, EV, wgt, host = _tree_with_tips(oracle, ntips, n, dtype, 9, coded)
    esums, escal = oracle.traverse(4, 4, ops, host, pm, EV, n, wgt, want_scalers=True)
    assert esums.sum() > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None if coded[t] else dev(dense[t]) for t in range(ntips)]
    clv += [torch.zeros(16 * n, dtype=tt, device="cuda") for _ in range(nslots - ntips)]
    tips = [dev(codes[t]) if coded[t] else None for t in range(ntips)] + [None] * (nslots - ntips)
    sums = torch.zeros(ops.shape[0], dtype=torch.int64, device="cuda")
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(ops.shape[0])]
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, tips=tips)
    torch.cuda.synchronize()
    for s in range(ntips, nslots):
        assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
    assert np.array_equal(sums.cpu().numpy(), esums)
    for j in range(ops.shape[0]):
        assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j


def test_caterpillar_inner_tip(ctx, oracle):
    """Caterpillar ((((t0,t1),t2),t3),t4): every op after the first is
    inner/tip, run as tip/inner with the children and matrices swapped."""
    import torch

    n = 1000
    rng = np.random.default_rng(21)
    codes = [oracle.random_tip_codes(rng, n, 0.3) for _ in range(5)]
    ops = np.array([[5, 0, 1, 0], [6, 5, 2, 1], [7, 6, 3, 2], [8, 7, 4, 3]], np.int32)
    pm = rng.random(4 * 128) * 0.5
    EV = rng.random(16)
    host = [oracle.expand_tips(c) for c in codes] + [np.zeros(16 * n) for _ in range(4)]
    esums, _ = oracle.traverse(4, 4, ops, host, pm, EV, n)
    clv = [None] * 5 + [torch.zeros(16 * n, dtype=torch.float64, device="cuda") for _ in range(4)]
    tips = [dev(c) for c in codes] + [None] * 4
    sums = torch.zeros(4, dtype=torch.int64, device="cuda")
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, None, None, sums, tips=tips)
    torch.cuda.synchronize()
    for s in range(5, 9):
        assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
    assert np.array_equal(sums.cpu().numpy(), esums)


def test_tips_reject_bad_args(ctx):
    import plfx
    import torch

    n = 16
    z = torch.zeros(16 * n, dtype=torch.float64, device="cuda")
    t = torch.zeros(n, dtype=torch.uint8, device="cuda")
    m = torch.zeros(64, dtype=torch.float64, device="cuda")
    x3 = torch.zeros(16 * n, dtype=torch.float64, device="cuda")
    with pytest.raises(plfx.PlfxError):   # both tip and CLV for child 1
        ctx.plf_tips_dev(x3, m[:16], n, m, m, x1=z, tip1=t, x2=z)
    with pytest.raises(plfx.PlfxError):   # neither for child 2
        ctx.plf_tips_dev(x3, m[:16], n, m, m, tip1=t)
    with pytest.raises(plfx.PlfxError):   # a tip slot as parent
        ctx.traverse(np.array([[0, 1, 2, 0]], np.int32), [None, z, z], torch.zeros(128, dtype=torch.float64,
                     device="cuda"), m[:16], n, tips=[t, None, None])


def test_tree64_tips_full_size_window(ctx, oracle):
    """BASELINE config 3 with coded tips: 64 taxa, 2^20 sites, f64; a 4096-site
    window checked bit-exactly against the oracle on the expanded window."""
    import torch

    n = 1 << 20
    ntips = 64
    ops = oracle.balanced_tree_ops(ntips)
    nslots = ntips + ops.shape[0]
    g = torch.Generator(device="cuda")
    g.manual_seed(20250117)
    tips = [torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device="cuda")[
        torch.randint(0, 4, (n,), device="cuda", generator=g)] for _ in range(ntips)]
    tips += [None] * (nslots - ntips)
    clv = [None] * ntips + [torch.empty(16 * n, dtype=torch.float64, device="cuda")
                            for _ in range(nslots - ntips)]
    pm = torch.rand(ops.shape[0] * 128, dtype=torch.float64, device="cuda", generator=g) * 0.25
    EV = torch.rand(16, dtype=torch.float64, device="cuda", generator=g) * 0.25
    sums = torch.zeros(ops.shape[0], dtype=torch.int64, device="cuda")
    ctx.traverse(ops, clv, pm, EV, n, None, None, sums, tips=tips)
    torch.cuda.synchronize()
    lo, m = 700_001, 4096
    win = [oracle.expand_tips(t[lo:lo + m].cpu().numpy()) for t in tips[:ntips]]
    win += [np.zeros(16 * m) for _ in range(nslots - ntips)]
    oracle.traverse(4, 4, ops, win, pm.cpu().numpy(), EV.cpu().numpy(), m)
    for s in range(ntips, nslots):
        assert np.array_equal(bits(clv[s][16 * lo:16 * (lo + m)].cpu().numpy()), bits(win[s])), s
    assert int(sums.sum().item()) > 0
