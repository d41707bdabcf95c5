"""GPU tests of the S=20 (protein) kernel, BASELINE configs[4].  The reference
is DNA-only: parity is against the oracle's generic restatement of
the same loop (plfo_plf_gen_*), which reproduces the pinned DNA plf()
bit-for-bit at S=4, and -- on the embedded 4-state sub-space (a DNA problem in
states 0..3 of 20, tests/test_protein_embedded.py) -- against the reference's
own plf(): test_protein_embedded_dna_*.  EXACT mode: bit-identical; FMA mode:
within 1e-12 relative (one rounding per fused term), identical scaler
decisions."""
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


def run(ctx, x1, x2, EV, left, right, w, n, fma, valu=False):
    import torch

    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    x3 = torch.empty(V * n, dtype=t[0].dtype, device="cuda")
    sc = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, t[5], sc, s, n=n, fma=fma, valu=valu)
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
    """FMA mode (f64: v_mfma_f64_16x16x4 / 4x4x4, f32: v_mfma_f32_16x16x4 with
    rows 16..19 on 4x4x1_16b and permlane transposes -- all k-ordered fma
    chains) is bit-identical to the oracle's fma() restatement and within
    1e-12 (f64) of the unfused loop."""
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


@pytest.mark.parametrize("fma", [False, True])
def test_protein_f32_many_trips(ctx, oracle, fma):
    """f32 at 2^16 + 1 sites (every block runs several trips through the tile
    prefetch, and the last tile is ragged): FMA mode on the matrix cores
    (plf_prot_mfma32_kernel) bit-identical to the oracle's fmaf restatement,
    exact mode (plf_prot_lds_kernel<float>) to plf()'s loop; scaler bytes and
    the weighted sum exact."""
    n = (1 << 16) + 1
    x1, x2, EV, left, right, w = gen(n, np.float32, 77)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=fma)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=fma)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc and esc.sum() > 0


@pytest.mark.parametrize("fma", [False, True])
def test_protein_f64_many_trips(ctx, oracle, fma):
    """f64 at 3 x 2^16 + 5 sites (six trips per block at the co-resident grid,
    the last tile ragged; weights 0..3): the exact kernel loads each site's
    weight at the top of the trip (plf_prot.hpp prot_lds_body), the FMA kernel
    inside the scaled-site branch -- both give plf()'s (resp. the fma
    restatement's) CLVs bit for bit and the exact weighted scaler sum."""
    n = 3 * (1 << 16) + 5
    x1, x2, EV, left, right, w = gen(n, np.float64, 78)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=fma)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=fma)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc and esc.sum() > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [4099, 3 * (1 << 15) + 7])
def test_protein_batched_nodes(ctx, oracle, dtype, n):
    """Several protein nodes in one batched launch (plf_prot_lds_batch_kernel:
    node = blockIdx.y, each node with its own grid stride and sum workspace):
    every node's CLV, scaler bytes and weighted sum bit-exact vs plf()'s loop,
    nodes with and without a scaler-sum output mixed in one launch."""
    import torch

    nodes, exp = [], []
    EV = None
    for k in range(5):
        x1, x2, ev, left, right, w = gen(n, dtype, 90 + k)
        if EV is None:
            EV, wgt = ev, w
        e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, wgt)
        nd = {"x1": dev(x1), "x2": dev(x2), "left": dev(left), "right": dev(right),
              "x3": torch.empty(V * n, dtype=torch.float64 if dtype == np.float64 else torch.float32,
                                device="cuda"),
              "scaler": torch.empty(n, dtype=torch.uint8, device="cuda")}
        if k != 2:
            nd["scaler_sum"] = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        nodes.append(nd)
        exp.append((e3, esc, einc))
    ctx.plf_batch_dev(nodes, dev(EV), n, dev(wgt), states=S)
    torch.cuda.synchronize()
    for k, (nd, (e3, esc, einc)) in enumerate(zip(nodes, exp)):
        assert np.array_equal(bits(nd["x3"].cpu().numpy()), bits(e3)), k
        assert np.array_equal(nd["scaler"].cpu().numpy(), esc), k
        if "scaler_sum" in nd:
            assert int(nd["scaler_sum"].item()) == einc, k
    assert sum(e[2] for e in exp) > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_protein_batched_level_fma(ctx, oracle, dtype):
    """A 4-taxon protein tree in FMA mode: its first level (two nodes) runs as
    one batched launch of the matrix-core kernel (plf_prot_mfma(32)_batch_kernel),
    the root as a one-node launch; every node bit-exact vs the oracle's fma()
    restatement applied node by node, scaler sums exact."""
    import torch

    n, ntips = (1 << 16) + 3, 4
    rng = np.random.default_rng(11)
    ops = oracle.balanced_tree_ops(ntips)
    nops = ops.shape[0]
    tips = [rng.random(V * n).astype(dtype) for _ in range(ntips)]
    tips[0].reshape(n, V)[0::4] *= 1e-14
    pm = rng.random(nops * 2 * CAT * S * S).astype(dtype)
    EV = (rng.random(S * S) - 0.25).astype(dtype)
    wgt = rng.integers(0, 4, n).astype(np.int32)
    host = [t.copy() for t in tips] + [None] * nops
    esums = []
    for j, (p, c1, c2, m) in enumerate(ops):
        L = pm[(2 * m) * CAT * S * S:(2 * m + 1) * CAT * S * S]
        R = pm[(2 * m + 1) * CAT * S * S:(2 * m + 2) * CAT * S * S]
        e3, _, einc = oracle.plf_generic(S, CAT, host[c1], host[c2], EV, L, R, wgt, fma=True)
        host[p] = e3
        esums.append(einc)
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [dev(t) for t in tips] + [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), None, sums, states=S, fma=True)
    torch.cuda.synchronize()
    for s_ in range(ntips, ntips + nops):
        assert np.array_equal(bits(clv[s_].cpu().numpy()), bits(host[s_])), s_
    assert sums.cpu().numpy().tolist() == esums and sum(esums) > 0


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


@pytest.fixture
def small_grid_ctx(monkeypatch):
    """A context whose grid-stride kernels launch 3 blocks (PLFX_MAX_BLOCKS):
    a few thousand sites then give every block dozens of trips."""
    import plfx

    monkeypatch.setenv("PLFX_MAX_BLOCKS", "3")
    c = plfx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("kind", ["dense", "tip1", "tip2", "both"])
def test_protein_f64_fma_tile_queue(small_grid_ctx, oracle, kind):
    """The f64 FMA kernel's device-wide tile queue (kDyn: from 32 tiles per
    block; here 3 blocks, 121 tiles, a ragged last one): bit-identical to the
    oracle's fused restatement on the expanded CLVs, scaler bytes and sum exact,
    three launches in a row (the queue words reset themselves).  Both-tip nodes
    keep the fixed stride."""
    import torch

    ctx = small_grid_ctx
    n = 3 * 64 * 40 + 37
    rng = np.random.default_rng(321)
    x1, x2, EV, left, right, w = gen(n, np.float64, 99)
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1 = oracle.expand_protein_tips(c1, np.float64) if kind in ("tip1", "both") else x1
    e2 = oracle.expand_protein_tips(c2, np.float64) if kind in ("tip2", "both") else x2
    f3, fsc, finc = oracle.plf_generic(S, CAT, e1, e2, EV, left, right, w, fma=True)
    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    for rep in range(3):
        x3 = torch.full((V * n,), float("nan"), dtype=torch.float64, device="cuda")
        sc = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        if kind == "dense":
            ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, t[5], sc, s, n=n, fma=True)
        else:
            kw = dict(x1=t[0]) if kind == "tip2" else dict(tip1=dev(c1))
            kw.update(x2=t[1]) if kind == "tip1" else kw.update(tip2=dev(c2))
            ctx.plf_tips_dev(x3, t[2], n, t[3], t[4], wgt=t[5], scaler=sc, scaler_sum=s, states=S,
                             fma=True, **kw)
        torch.cuda.synchronize()
        assert np.array_equal(bits(x3.cpu().numpy()), bits(f3)), rep
        assert np.array_equal(sc.cpu().numpy(), fsc) and int(s.item()) == finc, rep


def test_protein_f64_fma_tile_queue_full_grid(ctx, oracle):
    """2^20 + 37 sites at the default grid (512 blocks: 32 tiles per block and
    more, the queue path) and then 2^18 (the fixed stride) on the same stream:
    bit-identical to the oracle's fused restatement, sums exact."""
    for n in ((1 << 20) + 37, 1 << 18):
        x1, x2, EV, left, right, w = gen(n, np.float64, 1234 + n)
        x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=True)
        f3, fsc, finc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
        assert np.array_equal(bits(x3), bits(f3))
        assert np.array_equal(sc, fsc) and s == finc and fsc.sum() > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_protein_traverse_exact(ctx, oracle, dtype):
    """Protein traversal (states=20, one launch per node): CLVs, scaler bytes
    and sums bit-exact vs the oracle's sequential traversal; the FMA-mode
    traversal's root lnL within 1e-10 of the exact one (lnL is invariant to
    where the rescales happen)."""
    import torch

    n, ntips = 513, 8
    rng = np.random.default_rng(3)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    tips = [rng.random(V * n).astype(dtype) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.01).astype(dtype)  # deep levels underflow
    EV = (rng.random(S * S) * 0.01).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [t.copy() for t in tips] + [np.zeros(V * n, dtype) for _ in range(nops)]
    esums, escal = oracle.traverse(S, CAT, ops, host, pm, EV, n, wgt, want_scalers=True)
    assert esums.sum() > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    lnl = {}
    for fma in (False, True) if dtype == np.float64 else (False,):
        clv = [dev(t) for t in tips] + [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
        sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
        scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
        ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, states=S, fma=fma)
        out = torch.zeros(1, dtype=torch.float64, device="cuda")
        ctx.root_lnl(clv[-1], n, out, wgt=dev(wgt), scaler_sums=sums, states=S)
        torch.cuda.synchronize()
        lnl[fma] = float(out.item())
        if not fma:
            for s in range(ntips, nslots):
                assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
            assert np.array_equal(sums.cpu().numpy(), esums)
            for j in range(nops):
                assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j
    if True in lnl:
        assert abs(lnl[True] - lnl[False]) <= 1e-10 * abs(lnl[False])


def test_protein_model_pipeline_lnl(ctx, oracle):
    """A 20-state reversible model end to end: eigensystem -> device P
    matrices (states=20) -> protein traversal -> root lnL, against an
    independent numpy pruning with scipy.linalg.expm (1e-10 relative)."""
    import plfx
    import torch
    from scipy.linalg import expm

    n, ntips = 400, 8
    rng = np.random.default_rng(20)
    exch = rng.random(S * (S - 1) // 2) * 2 + 0.1
    freqs = rng.random(S) + 0.2
    pi = freqs / freqs.sum()
    R = np.zeros((S, S))
    R[np.triu_indices(S, 1)] = exch
    R = R + R.T
    Q = R * pi[None, :]
    np.fill_diagonal(Q, -Q.sum(axis=1))
    Q /= -(pi * np.diag(Q)).sum()
    e = plfx.model_eigen(exch, freqs)
    rates = plfx.gamma_rates(0.8, CAT)
    ops = oracle.balanced_tree_ops(ntips)
    nops = ops.shape[0]
    blen = rng.random(2 * nops) * 0.4 + 0.02
    obs = [rng.integers(0, S, n) for _ in range(ntips)]
    tipx = []
    for o in obs:  # one observed amino acid per site: indicator in every category
        x = np.zeros((n, CAT, S))
        x[np.arange(n), :, o] = 1.0
        tipx.append(x)
    clvs = {t: (tipx[t], np.zeros(n)) for t in range(ntips)}
    for p, c1, c2, m in ops:
        out = None
        for child, bl in ((c1, blen[2 * m]), (c2, blen[2 * m + 1])):
            u = np.stack([clvs[child][0][:, c, :] @ expm(Q * rates[c] * bl).T for c in range(CAT)], axis=1)
            out = u if out is None else out * u
        mx = out.reshape(n, -1).max(axis=1)
        clvs[p] = (out / mx[:, None, None], clvs[c1][1] + clvs[c2][1] + np.log(mx))
    root, logs = clvs[ops[-1][0]]
    exp_lnl = float(np.sum(np.log(np.einsum("c,ncs,s->n", np.full(CAT, 1 / CAT), root, pi)) + logs))

    pm = torch.empty(2 * nops * CAT * S * S, dtype=torch.float64, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(blen), pm, states=S, convention=plfx.PMAT_STATE)
    EVd = dev(plfx.model_ev(e, S, plfx.PMAT_STATE))
    clv = [dev(x.reshape(-1)) for x in tipx] + [torch.zeros(V * n, dtype=torch.float64, device="cuda")
                                                for _ in range(nops)]
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
    ctx.traverse(ops, clv, pm, EVd, n, None, None, sums, states=S, fma=True)
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    ctx.root_lnl(clv[-1], n, out, freq=dev(pi), scaler_sums=sums, states=S)
    torch.cuda.synchronize()
    got = float(out.item())
    assert abs(got - exp_lnl) <= 1e-10 * abs(exp_lnl), (got, exp_lnl)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("kind", ["tip1", "tip2", "both"])
@pytest.mark.parametrize("n", [1, 65, 3001])
def test_protein_tip_children(ctx, oracle, dtype, fma, kind, n):
    """Protein tips (uint8 code indices into the 24-row table: one amino acid,
    B, Z, X, gap, junk >= 24): bit-identical to the same mode's computation on
    the expanded dense CLVs (the oracle's restatement, exact or fma)."""
    import torch

    rng = np.random.default_rng(77 + n)
    x1, x2, EV, left, right, w = gen(n, dtype, 11 + n)
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1 = oracle.expand_protein_tips(c1, dtype) if kind in ("tip1", "both") else x1
    e2 = oracle.expand_protein_tips(c2, dtype) if kind in ("tip2", "both") else x2
    f3, fsc, finc = oracle.plf_generic(S, CAT, e1, e2, EV, left, right, w, fma=fma)
    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    x3 = torch.empty(V * n, dtype=t[0].dtype, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    kw = dict(x1=t[0]) if kind == "tip2" else dict(tip1=dev(c1))
    kw.update(x2=t[1]) if kind == "tip1" else kw.update(tip2=dev(c2))
    ctx.plf_tips_dev(x3, t[2], n, t[3], t[4], wgt=t[5], scaler=sc, scaler_sum=s, states=S,
                     fma=fma, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
    assert np.array_equal(sc.cpu().numpy(), fsc) and int(s.item()) == finc


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kind", ["tip1", "tip2", "both"])
def test_protein_tip_children_many_trips(ctx, oracle, dtype, kind):
    """The matrix-core (FMA) kernels' tip paths across many trips per block
    (2^16 + 1 sites: every block loops, and the next trip's dense tile is
    fetched while the current one is multiplied), bit-identical to
    the oracle's fused restatement on the expanded CLVs."""
    test_protein_tip_children(ctx, oracle, dtype, True, kind, (1 << 16) + 1)


def test_protein_tip_vector_table(ctx, oracle):
    """A caller tip-vector table (24 x 20, e.g. eigen coordinates or a
    different ambiguity model) replaces the default one."""
    import torch

    n = 777
    rng = np.random.default_rng(5)
    x1, x2, EV, left, right, w = gen(n, np.float64, 9)
    tv = rng.random((oracle.PROT_CODES, S)) - 0.3
    c1 = oracle.random_protein_codes(rng, n, 0.5)
    e1 = oracle.expand_protein_tips(c1, np.float64, tipvec=tv)
    f3, fsc, finc = oracle.plf_generic(S, CAT, e1, x2, EV, left, right, w)
    x3 = torch.empty(V * n, dtype=torch.float64, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_tips_dev(x3, dev(EV), n, dev(left), dev(right), tip1=dev(c1), x2=dev(x2), wgt=dev(w),
                     scaler_sum=s, tipvec=dev(tv), states=S)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(f3)) and int(s.item()) == finc


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_protein_traverse_with_tips(ctx, oracle, dtype):
    """Protein tree with coded tips (a mix of coded and dense leaves): the
    exact traversal is bit-exact against the oracle's sequential traversal on
    the expanded leaves; the FMA traversal's root lnL is within 1e-10."""
    import torch

    n, ntips = 700, 16
    rng = np.random.default_rng(8)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    coded = [t % 3 != 2 for t in range(ntips)]
    codes = [oracle.random_protein_codes(rng, n, 0.2) for _ in range(ntips)]
    dense = [rng.random(V * n).astype(dtype) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.05).astype(dtype)
    EV = (rng.random(S * S) * 0.05).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_protein_tips(codes[t], dtype) if coded[t] else dense[t].copy()
            for t in range(ntips)] + [np.zeros(V * n, dtype) for _ in range(nops)]
    esums, escal = oracle.traverse(S, CAT, ops, host, pm, EV, n, wgt, want_scalers=True)
    assert esums.sum() > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    lnl = {}
    for fma in (False, True) if dtype == np.float64 else (False,):
        clv = [None if coded[t] else dev(dense[t]) for t in range(ntips)]
        clv += [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
        tips = [dev(codes[t]) if coded[t] else None for t in range(ntips)] + [None] * nops
        sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
        scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
        ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, tips=tips, states=S,
                     fma=fma)
        out = torch.zeros(1, dtype=torch.float64, device="cuda")
        ctx.root_lnl(clv[-1], n, out, wgt=dev(wgt), scaler_sums=sums, states=S)
        torch.cuda.synchronize()
        lnl[fma] = float(out.item())
        if not fma:
            for s in range(ntips, nslots):
                assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
            assert np.array_equal(sums.cpu().numpy(), esums)
            for j in range(nops):
                assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j
    if True in lnl:
        assert abs(lnl[True] - lnl[False]) <= 1e-10 * abs(lnl[False])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
def test_protein_signed_zero_inputs(ctx, oracle, dtype, fma):
    """Inputs full of +-0.0, negative matrix entries and underflowing products:
    the exact kernels start their ump chains at the first product (plf_dna.hpp,
    site_cat) and still equal the oracle's plf() order bit for bit; FMA mode
    equals the fma() restatement."""
    rng = np.random.default_rng(5)
    n = 1000

    def field(size):
        v = (rng.random(size) - 0.5).astype(dtype)
        r = rng.random(size)
        v[r < 0.3] = dtype(0.0)
        v[(r >= 0.3) & (r < 0.5)] = dtype(-0.0)
        v[(r >= 0.5) & (r < 0.55)] *= np.finfo(dtype).tiny
        return v

    x1, x2, EV, left, right = field(V * n), field(V * n), field(S * S), field(CAT * S * S), field(CAT * S * S)
    w = rng.integers(0, 4, n).astype(np.int32)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=fma)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=fma)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc


@pytest.mark.parametrize("tips", [False, True])
def test_bench_prottree64_small(tips):
    """bench.py --workload prottree64 end to end at a small size: the level-
    batched protein tree sweep + root lnL runs, rescales (scaler events > 0),
    and its first node matches the oracle bit for bit (cpu_baseline check)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, str(root / "bench.py"), "--workload", "prottree64", "--sites", "4099",
           "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.2", "--no-second-region"] + \
        (["--tips"] if tips else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(root))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["check"] == "ok" and d["cpu_baseline"]["check"] == "ok", d
    assert d["config"]["scaler_events"] > 0 and d["config"]["nodes_per_gpu_per_step"] == 63


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_protein_root_lnl_tiles(ctx, oracle, dtype):
    """The protein root lnL (root_lnl_prot_kernel: 64-site LDS tiles, wave =
    category) at a multi-trip, ragged size with non-uniform category weights,
    frequencies, site weights and scaler totals: per-site log-likelihoods
    within 1e-15 of the oracle's (same L, libm vs device log) and the total
    within 1e-12."""
    import torch

    n = 3 * (1 << 16) + 11
    rng = np.random.default_rng(21)
    x = rng.random(V * n).astype(dtype)
    catw = rng.random(CAT)
    catw /= catw.sum()
    freq = rng.random(S)
    freq /= freq.sum()
    w = rng.integers(0, 4, n).astype(np.int32)
    sums = np.array([5, 0, 17], np.int64)
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    sl = torch.zeros(n, dtype=torch.float64, device="cuda")
    ctx.root_lnl(dev(x), n, out, catw=dev(catw), freq=dev(freq), wgt=dev(w), scaler_sums=dev(sums),
                 site_lnl=sl, states=S)
    torch.cuda.synchronize()
    exp, esl = oracle.root_lnl(S, CAT, x, n, catw=catw, freq=freq, wgt=w, scaler_sums=sums, site=True)
    got = sl.cpu().numpy()
    assert np.max(np.abs(got - esl) / np.maximum(np.abs(esl), 1e-300)) <= 1e-15
    assert abs(float(out.item()) - exp) <= 1e-12 * abs(exp)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("with_sum", [True, False])
@pytest.mark.parametrize("warm", [False, True])
def test_protein_tiptip_in_graph_capture(oracle, dtype, fma, with_sum, warm):
    """A tip/tip protein node captured in a HIP graph: whether or not the
    stream made a tip/tip call before (warm / cold), the capture holds the
    combination-table launch and the gather (2 kernel nodes: the tables come
    with the stream's workspace, nothing is allocated or waited for inside the
    capture).  Replays are bit-identical to the oracle, with and without the
    weighted sum."""
    import plfx
    import torch

    n = 5003
    rng = np.random.default_rng(31)
    _, _, EV, left, right, w = gen(n, dtype, 12)
    left = (left * 1e-11).astype(dtype)  # a mix of rescaled sites
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1, e2 = oracle.expand_protein_tips(c1, dtype), oracle.expand_protein_tips(c2, dtype)
    f3, fsc, finc = oracle.plf_generic(S, CAT, e1, e2, EV, left, right, w, fma=fma)
    assert 0 < fsc.sum() < n
    t = [dev(a) for a in (c1, c2, EV, left, right, w)]
    tt = torch.float64 if dtype == np.float64 else torch.float32
    x3 = torch.empty(V * n, dtype=tt, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda") if with_sum else None
    st = torch.cuda.Stream()
    ctx = plfx.Context(0)

    def call():
        ctx.plf_tips_dev(x3, t[2], n, t[3], t[4], tip1=t[0], tip2=t[1], wgt=t[5], scaler=sc,
                         scaler_sum=s, states=S, fma=fma, stream=st)

    torch.cuda.synchronize()
    if warm:
        call()
    else:  # the stream's workspace exists, its combination tables do not
        xd = dev(np.zeros(V * n, dtype))
        ctx.plf_tips_dev(x3, t[2], n, t[3], t[4], tip1=t[0], x2=xd, wgt=t[5], scaler=sc,
                         scaler_sum=s, states=S, fma=fma, stream=st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=st):
        call()
    from test_gpu_api import _kernel_nodes

    assert _kernel_nodes(g) == 2
    g.instantiate()
    for _ in range(2):
        x3.zero_()
        if s is not None:
            s.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
        assert np.array_equal(sc.cpu().numpy(), fsc)
        assert s is None or int(s.item()) == finc
    del g
    ctx.release_stream(st)
    ctx.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("with_sum", [True, False])
def test_protein_tiptip_level_in_graph_capture(oracle, dtype, fma, with_sum):
    """A 16-taxon all-coded protein tree traversed inside a capture on a
    stream whose only earlier call was a tip/dense node: its first level (8
    tip/tip nodes) goes through the combination tables of the stream's
    workspace (allocated with it) and the second level stages its children
    from them.  Replays equal a sequential oracle evaluation in the same mode
    bit for bit (CLVs, scaler bytes, sums)."""
    import plfx
    import torch

    n, ntips = 900, 16
    rng = np.random.default_rng(61)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    codes = [oracle.random_protein_codes(rng, n, 0.2) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.05).astype(dtype)
    EV = (rng.random(S * S) * 0.05).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_protein_tips(c, dtype) for c in codes] + [None] * nops
    M = CAT * S * S
    escal, einc = [], []
    for parent, a, b, p in ops:
        x3, sc, inc = oracle.plf_generic(S, CAT, host[a], host[b], EV, pm[2 * p * M:(2 * p + 1) * M],
                                         pm[(2 * p + 1) * M:(2 * p + 2) * M], wgt, fma=fma)
        host[parent] = x3
        escal.append(sc)
        einc.append(inc)
    assert sum(einc) > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None] * ntips + [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [dev(c) for c in codes] + [None] * nops
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda") if with_sum else None
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    pmd, EVd, wd = dev(pm), dev(EV), dev(wgt)
    st = torch.cuda.Stream()
    ctx = plfx.Context(0)
    # the stream's workspace: one tip/dense node first
    xd = torch.zeros(V * n, dtype=tt, device="cuda")
    ctx.plf_tips_dev(clv[ntips], EVd, n, pmd[:M], pmd[M:2 * M], tip1=tips[0], x2=xd, wgt=wd,
                     states=S, fma=fma, stream=st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        ctx.traverse(ops, clv, pmd, EVd, n, wd, scal, sums, tips=tips, states=S, fma=fma, stream=st)
    for _ in range(2):
        for x in clv[ntips:]:
            x.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for s_ in range(ntips, nslots):
            assert np.array_equal(bits(clv[s_].cpu().numpy()), bits(host[s_])), s_
        for j in range(nops):
            assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j
        if sums is not None:
            assert sums.cpu().tolist() == einc
    del g
    ctx.release_stream(st)
    ctx.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 129])
def test_protein_tiptip_edge_sizes(ctx, oracle, dtype, fma, n):
    """Tip/tip protein nodes (combination tables + gather) at ragged sizes
    around the 64-site tile, with and without weights and per-site scaler
    output, junk codes >= 24 included: the same values as the oracle on the
    expanded leaves (exact: bit for bit; FMA: the fused restatement)."""
    import torch

    rng = np.random.default_rng(900 + n)
    _, _, EV, left, right, w = gen(n, dtype, 40 + n)
    left = (left * 1e-10).astype(dtype)  # code pairs on both sides of the 2^-32 rescale threshold
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    c1[0] = 200  # junk code: the all-ones row
    e1, e2 = oracle.expand_protein_tips(c1, dtype), oracle.expand_protein_tips(c2, dtype)
    for wgt in (None, w):
        ww = np.ones(n, np.int32) if wgt is None else wgt
        f3, fsc, finc = oracle.plf_generic(S, CAT, e1, e2, EV, left, right, ww, fma=fma)
        for with_scaler in (False, True):
            x3 = torch.empty(V * n, dtype=torch.float64 if dtype == np.float64 else torch.float32,
                             device="cuda")
            sc = torch.empty(n, dtype=torch.uint8, device="cuda") if with_scaler else None
            s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
            ctx.plf_tips_dev(x3, dev(EV), n, dev(left), dev(right), tip1=dev(c1), tip2=dev(c2),
                             wgt=None if wgt is None else dev(wgt), scaler=sc, scaler_sum=s,
                             states=S, fma=fma)
            torch.cuda.synchronize()
            assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
            assert int(s.item()) == finc
            if with_scaler:
                assert np.array_equal(sc.cpu().numpy(), fsc)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_protein_traverse_all_coded_128(ctx, oracle, dtype):
    """A 128-taxon protein tree with every leaf coded: its first level is 64
    tip/tip nodes, two batches of 32 through the same stream's combination
    tables (the second batch overwrites the first's tables in stream order).
    Exact traversal bit for bit against the oracle's sequential traversal."""
    import torch

    n, ntips = 300, 128
    rng = np.random.default_rng(128)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    codes = [oracle.random_protein_codes(rng, n, 0.2) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.05).astype(dtype)
    EV = (rng.random(S * S) * 0.05).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_protein_tips(codes[t], dtype) for t in range(ntips)]
    host += [np.zeros(V * n, dtype) for _ in range(nops)]
    esums, escal = oracle.traverse(S, CAT, ops, host, pm, EV, n, wgt, want_scalers=True)
    assert esums.sum() > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None] * ntips + [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [dev(c) for c in codes] + [None] * nops
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, tips=tips, states=S)
    torch.cuda.synchronize()
    for s in range(ntips, nslots):
        assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
    assert np.array_equal(sums.cpu().numpy(), esums)
    for j in range(nops):
        assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [True, False])
@pytest.mark.parametrize("with_sum", [True, False])
@pytest.mark.parametrize("ntips", [32, 128])
def test_protein_coded_tree_table_children(ctx, oracle, dtype, fma, with_sum, ntips):
    """Protein tree (f64, f32; FMA or exact), every leaf coded: the second level's nodes stage
    their children's tiles from the first level's combination tables
    (plf_prot_mfma_tab_batch_kernel) -- at 128 taxa only the second table
    group's parents can (the first group's tables are overwritten), the rest
    read the children's CLVs.  Every CLV, scaler byte and sum equals a
    sequential evaluation by the oracle's fused loop bit for bit."""
    import torch

    n = 1500
    rng = np.random.default_rng(ntips + 3)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    codes = [oracle.random_protein_codes(rng, n, 0.2) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.05).astype(dtype)
    EV = (rng.random(S * S) * 0.05).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_protein_tips(c, dtype) for c in codes] + [None] * nops
    M = CAT * S * S
    escal, einc = [], []
    for parent, a, b, p in ops:
        x3, sc, inc = oracle.plf_generic(S, CAT, host[a], host[b], EV, pm[2 * p * M:(2 * p + 1) * M],
                                         pm[(2 * p + 1) * M:(2 * p + 2) * M], wgt, fma=fma)
        host[parent] = x3
        escal.append(sc)
        einc.append(inc)
    assert sum(einc) > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None] * ntips + [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [dev(c) for c in codes] + [None] * nops
    sums = torch.full((nops,), -1, dtype=torch.int64, device="cuda") if with_sum else None
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, tips=tips, states=S, fma=fma)
    torch.cuda.synchronize()
    for s_ in range(ntips, nslots):
        assert np.array_equal(bits(clv[s_].cpu().numpy()), bits(host[s_])), s_
    for j in range(nops):
        assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j
    if with_sum:
        assert sums.cpu().tolist() == einc


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [1, 4099, 65537])
def test_protein_embedded_dna_node_equals_reference(ctx, oracle, dtype, n):
    """The protein exact kernels pinned by the reference itself on the embedded
    4-state sub-space (oracle.embed_dna_*, tests/test_protein_embedded.py): a
    DNA node in states 0..3 of 20 gives states 0..3 equal to the reference's
    plf() (oracle/_ref: the f32 build / the double instantiation) bit for bit,
    states 4..19 exactly +0.0, and the reference's scaler bytes and sum."""
    if not oracle.ref_available(dtype):
        pytest.skip("oracle/_ref not shipped")
    d = oracle.gen_hostmem(n, dtype, 500 + n)
    w = (np.arange(n, dtype=np.int32) % 5) - 1
    f = oracle._ref_call(dtype)
    r3 = np.empty(16 * n, dtype)
    rinc = f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w)
    rsc = oracle.ref_scaled_sites(f, d["x1"], d["x2"], d["EV"], d["left"], d["right"], n)
    x3, sc, s = run(ctx, oracle.embed_dna_clv(d["x1"]), oracle.embed_dna_clv(d["x2"]),
                    oracle.embed_dna_mats(d["EV"]), oracle.embed_dna_mats(d["left"]),
                    oracle.embed_dna_mats(d["right"]), w, n, fma=False)
    got, rest_zero = oracle.extract_dna_clv(x3)
    assert rest_zero
    assert np.array_equal(bits(got), bits(r3))
    assert np.array_equal(sc, rsc) and s == rinc


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("mode", ["dense", "coded", "mixed"])
def test_protein_embedded_dna_tree64_equals_reference_golden(ctx, oracle, dtype, mode):
    """configs[2]'s 64-taxon tree as a protein traversal (exact mode) on the
    embedded sub-space reproduces tests/golden/tree64.npz -- the reference's
    plf() composed per inner node -- byte for byte: batched level launches,
    and with coded leaves (DNA codes as protein codes into the embedded tip
    table) the tip/tip combination tables, their gather, tip/inner nodes and
    the parents that stage children from the tables."""
    import torch

    g = np.load(__import__("conftest").GOLDEN / "tree64.npz", allow_pickle=False)
    k = f"{'f32' if dtype == np.float32 else 'f64'}_{mode}"
    c = oracle.tree_golden_case(dtype, mode, int(g["n"]), int(g["seed"]))
    assert oracle.tree_case_digest(c) == str(g[f"{k}_inputs_sha256"])
    n, ops = c["n"], c["ops"]
    nops, nslots = ops.shape[0], 64 + ops.shape[0]
    codes = [None if cd is None else (cd & 15).astype(np.uint8) for cd in c["codes"]]
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None if cd is not None else dev(oracle.embed_dna_clv(t)) for t, cd in zip(c["tips"], codes)]
    clv += [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [None if cd is None else dev(cd) for cd in codes] + [None] * nops
    sums = torch.full((nops,), -7, dtype=torch.int64, device="cuda")
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    ctx.traverse(ops, clv, dev(oracle.embed_dna_mats(c["pm"])), dev(oracle.embed_dna_mats(c["EV"])), n,
                 dev(c["wgt"]), scal, sums, tips=tips, tipvec=dev(oracle.embedded_dna_tipvec(dtype)),
                 states=S, fma=False)
    torch.cuda.synchronize()
    digests = []
    for p in ops[:, 0]:
        x, rest_zero = oracle.extract_dna_clv(clv[int(p)].cpu().numpy())
        assert rest_zero, int(p)
        digests.append(oracle.clv_digest(x))
    bad = [j for j, (a, b) in enumerate(zip(digests, g[f"{k}_x3_sha256"])) if a != str(b)]
    assert not bad, f"parent CLVs of ops {bad[:8]} differ from the reference composition"
    assert np.array_equal(sums.cpu().numpy(), g[f"{k}_sums"])
    assert np.array_equal(np.stack([s_.cpu().numpy() for s_ in scal]), g[f"{k}_scaler"])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("n", [1, 4099, 65537])
def test_protein_fma_embedded_dna_node_equals_contracted_reference(ctx, oracle, dtype, n):
    """FMA mode (the configs[4] default: f64 16x16x4 + 4x4x4 matrix cores, f32
    16x16x4 + 4x4x1) on the embedded 4-state sub-space equals the reference
    source compiled with FMA contraction (oracle/_ref/libplfref{,_f64}_fma.so,
    every multiply-add of plf() fused in plf()'s order) bit for bit."""
    if not oracle.ref_available(dtype, "fma"):
        pytest.skip("oracle/_ref not shipped")
    d = oracle.gen_hostmem(n, dtype, 700 + n)
    w = (np.arange(n, dtype=np.int32) % 5) - 1
    f = oracle._ref_call(dtype, "fma")
    r3 = np.empty(16 * n, dtype)
    rinc = f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w)
    rsc = oracle.ref_scaled_sites(f, d["x1"], d["x2"], d["EV"], d["left"], d["right"], n)
    x3, sc, s = run(ctx, oracle.embed_dna_clv(d["x1"]), oracle.embed_dna_clv(d["x2"]),
                    oracle.embed_dna_mats(d["EV"]), oracle.embed_dna_mats(d["left"]),
                    oracle.embed_dna_mats(d["right"]), w, n, fma=True)
    got, rest_zero = oracle.extract_dna_clv(x3)
    assert rest_zero
    assert np.array_equal(bits(got), bits(r3))
    assert np.array_equal(sc, rsc) and s == rinc


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("mode", ["dense", "coded", "mixed"])
def test_protein_fma_embedded_tree64_equals_contracted_reference(ctx, oracle, dtype, mode):
    """The 64-taxon tree as an FMA-mode protein traversal on the embedded
    sub-space equals the FMA-contracted reference's plf() composed per inner
    node (oracle.ref_traverse over the fma build, live): every parent CLV,
    scaler byte and sum -- batched FMA levels, tip/tip tables and their
    gather, tip/inner nodes, table children."""
    import torch

    if not oracle.ref_available(dtype, "fma"):
        pytest.skip("oracle/_ref not shipped")
    g = np.load(__import__("conftest").GOLDEN / "tree64.npz", allow_pickle=False)
    c = oracle.tree_golden_case(dtype, mode, int(g["n"]), int(g["seed"]))
    n, ops = c["n"], c["ops"]
    nops = ops.shape[0]
    ref = [t.copy() for t in c["tips"]] + [np.zeros(16 * n, dtype) for _ in range(nops)]
    rsums, rscal = oracle.ref_traverse(ops, ref, c["pm"], c["EV"], n, c["wgt"], want_scalers=True, opt="fma")
    codes = [None if cd is None else (cd & 15).astype(np.uint8) for cd in c["codes"]]
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None if cd is not None else dev(oracle.embed_dna_clv(t)) for t, cd in zip(c["tips"], codes)]
    clv += [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [None if cd is None else dev(cd) for cd in codes] + [None] * nops
    sums = torch.full((nops,), -7, dtype=torch.int64, device="cuda")
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    ctx.traverse(ops, clv, dev(oracle.embed_dna_mats(c["pm"])), dev(oracle.embed_dna_mats(c["EV"])), n,
                 dev(c["wgt"]), scal, sums, tips=tips, tipvec=dev(oracle.embedded_dna_tipvec(dtype)),
                 states=S, fma=True)
    torch.cuda.synchronize()
    for j, p in enumerate(ops[:, 0]):
        x, rest_zero = oracle.extract_dna_clv(clv[int(p)].cpu().numpy())
        assert rest_zero, j
        assert np.array_equal(bits(x), bits(ref[int(p)])), j
        assert np.array_equal(scal[j].cpu().numpy(), rscal[j]), j
    assert np.array_equal(sums.cpu().numpy(), rsums)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("n", [4099, 65537])
def test_protein_five_dna_blocks_equal_reference(ctx, oracle, dtype, fma, n):
    """Five 4-state problems side by side in one protein node (states
    4b..4b+3, block-diagonal P and EV; oracle.embed_*_blocks) reach every state
    position of the protein kernels -- rows 16..19 go through the 4x4x4 (f64)
    / 4x4x1 (f32) matrix-core forms in FMA mode -- and each block equals its
    own reference plf(): the reference build in exact mode, the build with
    FMA contraction in FMA mode; scaler bytes and sum as the reference's (the
    blocks share the host_mem scaling pattern)."""
    opt = "fma" if fma else "O0"
    if not oracle.ref_available(dtype, opt):
        pytest.skip("oracle/_ref not shipped")
    ps = [oracle.gen_hostmem(n, dtype, 1200 + 7 * b + n % 97) for b in range(5)]
    w = (np.arange(n, dtype=np.int32) % 4) - 1
    f = oracle._ref_call(dtype, opt)
    refs, incs = [], []
    for d in ps:
        r3 = np.empty(16 * n, dtype)
        incs.append(f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w))
        refs.append(r3)
    rsc = oracle.ref_scaled_sites(f, ps[0]["x1"], ps[0]["x2"], ps[0]["EV"], ps[0]["left"], ps[0]["right"], n)
    x3, sc, s = run(ctx, oracle.embed_clv_blocks([d["x1"] for d in ps]),
                    oracle.embed_clv_blocks([d["x2"] for d in ps]),
                    oracle.embed_mat_blocks([d["EV"] for d in ps]),
                    oracle.embed_mat_blocks([d["left"] for d in ps]),
                    oracle.embed_mat_blocks([d["right"] for d in ps]), w, n, fma=fma)
    outs, rest_zero = oracle.extract_clv_blocks(x3, 5)
    assert rest_zero
    for b in range(5):
        assert np.array_equal(bits(outs[b]), bits(refs[b])), b
    assert len(set(incs)) == 1 and s == incs[0]
    assert np.array_equal(sc, rsc)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 257, 4097, 3 * (1 << 16) + 5, 1 << 18])
def test_protein_valu_fma_bits(ctx, oracle, n):
    """PLFX_FMA | PLFX_VALU (plf_prot_valu.hip: the LDS-tiled matvecs of the
    exact kernel with every multiply-add fused, BASELINE configs[4]'s "matvec,
    not MFMA"): bit-identical to the oracle's fma() restatement and to the
    matrix-core FMA kernel, scaler bytes and the weighted sum exact; ragged
    tiles, several trips per block and the full 2^18 size."""
    x1, x2, EV, left, right, w = gen(n, np.float64, 900 + n % 97)
    v3, vsc, vs = run(ctx, x1, x2, EV, left, right, w, n, fma=True, valu=True)
    m3, msc, ms = run(ctx, x1, x2, EV, left, right, w, n, fma=True)
    assert np.array_equal(bits(v3), bits(m3)) and np.array_equal(vsc, msc) and vs == ms
    f3, fsc, finc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    assert np.array_equal(bits(v3), bits(f3))
    assert np.array_equal(vsc, fsc) and vs == finc
    assert fsc.sum() > 0 or n < 4


@pytest.mark.parametrize("valu", [False, True])
def test_protein_f64_optional_outputs(ctx, oracle, valu):
    """The f64 FMA node without the scaler sum (and without scaler bytes or
    weights): the kernels' no-sum instantiations, matrix-core and VALU, give
    the same CLV bits and scaler bytes as with every output."""
    import torch

    n = 3001
    x1, x2, EV, left, right, w = gen(n, np.float64, 77)
    f3, fsc, _ = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    t = [dev(a) for a in (x1, x2, EV, left, right)]
    for wgt, with_sc in ((dev(w), True), (None, True), (None, False)):
        x3 = torch.empty(V * n, dtype=torch.float64, device="cuda")
        sc = torch.empty(n, dtype=torch.uint8, device="cuda") if with_sc else None
        ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, wgt, sc, None, n=n, fma=True, valu=valu)
        torch.cuda.synchronize()
        assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
        if with_sc:
            assert np.array_equal(sc.cpu().numpy(), fsc)


def test_protein_valu_fma_signed_zeros_and_flags(ctx, oracle):
    """The VALU FMA chains start from +0.0 as the fma() restatement does, on
    inputs full of +-0.0 and underflowing products; PLFX_VALU is refused
    in f32 and for DNA; in exact mode the same form gives plf()'s bits."""
    import torch

    import plfx

    rng = np.random.default_rng(11)
    n = 1000

    def field(size):
        v = rng.random(size) - 0.5
        r = rng.random(size)
        v[r < 0.3] = 0.0
        v[(r >= 0.3) & (r < 0.5)] = -0.0
        v[(r >= 0.5) & (r < 0.55)] *= np.finfo(np.float64).tiny
        return v

    x1, x2, EV, left, right = field(V * n), field(V * n), field(S * S), field(CAT * S * S), field(CAT * S * S)
    w = rng.integers(0, 4, n).astype(np.int32)
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=True, valu=True)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc
    # exact mode with the scalar-operand matrices: plf()'s loop bit for bit
    x3, sc, s = run(ctx, x1, x2, EV, left, right, w, n, fma=False, valu=True)
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
    assert np.array_equal(bits(x3), bits(e3))
    assert np.array_equal(sc, esc) and s == einc
    f = [dev(a.astype(np.float32)) for a in (x1, x2, EV, left, right)]
    with pytest.raises(plfx.PlfxError):
        ctx.plf_dev_gen(f[0], f[1], torch.empty_like(f[0]), f[2], f[3], f[4], S, fma=True, valu=True)
    d = [dev(a) for a in (x1[:16 * n], x2[:16 * n], EV[:16], left[:64], right[:64])]
    with pytest.raises(plfx.PlfxError):
        ctx.plf_dev_gen(d[0], d[1], torch.empty_like(d[0]), d[2], d[3], d[4], 4, fma=True, valu=True)


@pytest.mark.parametrize("n", [1, 63, 65, 4097, 3 * (1 << 16) + 5, 1 << 18])
def test_protein_valu_exact_bits(ctx, oracle, n):
    """The f64 exact node (plf_prot_valu_exact.hip: plf()'s separate
    roundings with the matrices as scalar operands, 3 waves per SIMD; the
    default for exact f64, PLFX_VALU or not): bit-identical to plf()'s double
    loop (the oracle) and to the LDS-matrix exact kernel, which still serves
    batched and tip nodes (one batched launch of this node below), scaler
    bytes and weighted sum exact."""
    import torch

    x1, x2, EV, left, right, w = gen(n, np.float64, 700 + n % 89)
    v3, vsc, vs = run(ctx, x1, x2, EV, left, right, w, n, fma=False, valu=True)
    d3, dsc, ds = run(ctx, x1, x2, EV, left, right, w, n, fma=False)
    assert np.array_equal(bits(v3), bits(d3)) and np.array_equal(vsc, dsc) and vs == ds
    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    l3 = torch.empty_like(t[0])
    lsc = torch.empty(n, dtype=torch.uint8, device="cuda")
    ls = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_batch_dev([dict(x1=t[0], x2=t[1], x3=l3, left=t[3], right=t[4], scaler=lsc, scaler_sum=ls)],
                      t[2], n, wgt=t[5], states=S)
    torch.cuda.synchronize()
    assert np.array_equal(bits(v3), bits(l3.cpu().numpy())) and np.array_equal(vsc, lsc.cpu().numpy())
    assert vs == int(ls.item())
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
    assert np.array_equal(bits(v3), bits(e3))
    assert np.array_equal(vsc, esc) and vs == einc
