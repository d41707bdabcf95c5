"""GPU tests of P-matrix generation (plfx.h section 9)
and of the whole likelihood pipeline built from it: GTR+Gamma4 eigensystem ->
device P matrices -> traversal (tips as state codes) -> root lnL, against an
independent numpy Felsenstein pruning that uses scipy.linalg.expm (the bar:
the north-star f64 tolerance, 1e-10 relative), and the reference's own AIE
stimuli -- a GTR + Gamma4 model's matrices and a four-taxon known-answer tree
-- reproduced through the device path (the last two tests)."""
import numpy as np
import pytest

import plfx
from scipy.linalg import expm

pytestmark = pytest.mark.gpu

LNL_RTOL = 1e-10


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gtr_q(exch, freqs):
    S = len(freqs)
    pi = np.asarray(freqs, float) / np.sum(freqs)
    R = np.zeros((S, S))
    R[np.triu_indices(S, 1)] = exch
    R = R + R.T
    Q = R * pi[None, :]
    np.fill_diagonal(Q, -Q.sum(axis=1))
    return Q / -(pi * np.diag(Q)).sum(), pi


@pytest.mark.parametrize("S", [4, 20])
@pytest.mark.parametrize("conv", [plfx.PMAT_STATE, plfx.PMAT_EIGEN])
def test_pmatrix_vs_expm(ctx, S, conv):
    import torch

    rng = np.random.default_rng(S + conv)
    exch = rng.random(S * (S - 1) // 2) * 2 + 0.05
    freqs = rng.random(S) + 0.1
    Q, pi = gtr_q(exch, freqs)
    e = plfx.model_eigen(exch, freqs)
    lam, V, Vi = e[:S], e[S:S + S * S].reshape(S, S), e[S + S * S:].reshape(S, S)
    rates = plfx.gamma_rates(0.7, 4)
    blen = np.concatenate([[0.0, 1e-6], rng.random(37) * 2, [10.0]])
    out = torch.empty(blen.size * 4 * S * S, dtype=torch.float64, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(blen), out, states=S, convention=conv)
    out32 = torch.empty(out.numel(), dtype=torch.float32, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(blen), out32, states=S, convention=conv)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(blen.size, 4, S, S)
    for b, t in enumerate(blen):
        for c in range(4):
            if conv == plfx.PMAT_STATE:
                exp_ = expm(Q * rates[c] * t)
                assert np.abs(got[b, c] - exp_).max() < 1e-12, (b, c)
            else:
                exp_ = V * np.exp(lam * rates[c] * t)[None, :]
                assert np.allclose(got[b, c], exp_, rtol=1e-13, atol=1e-15), (b, c)
    assert np.array_equal(out32.cpu().numpy(), out.cpu().numpy().astype(np.float32)) or \
        np.allclose(out32.cpu().numpy(), out.cpu().numpy(), rtol=2e-7, atol=1e-30)


def felsenstein_lnl(Q, pi, rates, catw, blen, ops, tipx, ntips, wgt):
    """Independent numpy pruning: CLVs (n, C, S) in state space, per-site
    log-scale kept separately, P = expm(Q r t)."""
    C = len(rates)
    clv = {t: (tipx[t], np.zeros(tipx[t].shape[0])) for t in range(ntips)}
    for p, c1, c2, m in ops:
        out = None
        logs = clv[c1][1] + clv[c2][1]
        for side, (child, bl) in enumerate(((c1, blen[2 * m]), (c2, blen[2 * m + 1]))):
            x = clv[child][0]
            u = np.stack([x[:, c, :] @ expm(Q * rates[c] * bl).T for c in range(C)], axis=1)
            out = u if out is None else out * u
        mx = out.reshape(out.shape[0], -1).max(axis=1)
        clv[p] = (out / mx[:, None, None], logs + np.log(mx))
    root, logs = clv[ops[-1][0]]
    site = np.einsum("c,ncs,s->n", catw, root, pi)
    return float(np.sum(wgt * (np.log(site) + logs)))


@pytest.mark.parametrize("conv,coded", [(plfx.PMAT_STATE, True), (plfx.PMAT_EIGEN, False),
                                        (plfx.PMAT_EIGEN, True)])
def test_gtr_gamma_pipeline_lnl(ctx, oracle, conv, coded):
    """GTR+G4 on a 16-taxon balanced tree, 5000 sites: device P matrices ->
    traverse -> root lnL equals the numpy pruning within 1e-10 relative.
    STATE: tips as uint8 state codes, EV = I.  EIGEN: tips as dense eigen-
    coordinate CLVs Vinv.bits, EV = Vinv^T, root weights pi.V.  EIGEN_CODED:
    the eigen convention with coded tips and the eigen tip-vector table."""
    import torch

    rng = np.random.default_rng(31 + conv)
    n, ntips = 5000, 16
    exch = np.array([1.2, 3.9, 0.8, 1.1, 4.6, 1.0])
    freqs = np.array([0.31, 0.19, 0.22, 0.28])
    Q, pi = gtr_q(exch, freqs)
    e = plfx.model_eigen(exch, freqs)
    Vi = e[4 + 16:].reshape(4, 4)
    rates = plfx.gamma_rates(0.42, 4)
    catw = np.full(4, 0.25)
    ops = oracle.balanced_tree_ops(ntips)
    nops = ops.shape[0]
    blen = rng.random(2 * nops) * 0.3 + 0.01
    codes = [oracle.random_tip_codes(rng, n, 0.05) for _ in range(ntips)]
    codes = [np.where((c & 15) == 0, 15, c).astype(np.uint8) for c in codes]  # no empty sets
    wgt = rng.integers(1, 4, n).astype(np.int32)
    tipx = [oracle.expand_tips(c).reshape(n, 4, 4) for c in codes]
    exp_lnl = felsenstein_lnl(Q, pi, rates, catw, blen, ops, tipx, ntips, wgt)

    pm = torch.empty(2 * nops * 64, dtype=torch.float64, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(blen), pm, states=4, convention=conv)
    EV = dev(plfx.model_ev(e, 4, conv))
    nslots = ntips + nops
    clv = [torch.empty(16 * n, dtype=torch.float64, device="cuda") for _ in range(nops)]
    tipvec = None
    if coded:
        tips = [dev(c) for c in codes] + [None] * nops
        clv = [None] * ntips + clv
        if conv == plfx.PMAT_EIGEN:
            tipvec = dev(plfx.model_tip_vectors(e, conv))
    else:
        tips = None
        clv = [dev(np.einsum("ls,ncs->ncl", Vi, x).reshape(-1)) for x in tipx] + clv
    sums = torch.zeros(nops, dtype=torch.int64, device="cuda")
    ctx.traverse(ops, clv, pm, EV, n, dev(wgt), None, sums, tips=tips, tipvec=tipvec)
    w = dev(plfx.model_root_weights(e, freqs, conv))
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    ctx.root_lnl(clv[nslots - 1], n, out, catw=dev(catw), freq=w, wgt=dev(wgt), scaler_sums=sums)
    torch.cuda.synchronize()
    got = float(out.item())
    assert abs(got - exp_lnl) <= LNL_RTOL * abs(exp_lnl), (got, exp_lnl)


def test_pmatrix_rejects_bad_args(ctx):
    import torch

    e = dev(plfx.model_eigen(np.ones(6), np.full(4, 0.25)))
    r = dev(np.ones(4))
    b = dev(np.ones(3))
    out = torch.empty(3 * 64, dtype=torch.float64, device="cuda")
    with pytest.raises(plfx.PlfxError):
        ctx.pmatrix(e, r, b, out, convention=7)
    with pytest.raises(plfx.PlfxError):
        ctx.pmatrix(e, r, b, out[:10])


def test_device_pmatrix_reproduces_reference_aie_matrices(ctx):
    """The device P-matrix path with the generator parameters recovered from
    the reference's AIE stimuli (tests/test_model.py, aie/data/inputEV0.txt,
    inputbranchleft{0..3}.txt): STATE matrices equal the data's state-space
    transition matrices to its six printed decimals, and the EIGEN matrices
    with the library's EV compose to the same STATE matrices (the eigenvector
    basis drops out)."""
    import torch

    from test_model import AIE_ALPHA, AIE_EXCH, AIE_T, aie_model

    EV, Pe, Ps = aie_model()
    e = plfx.model_eigen(AIE_EXCH, EV[:, 0])
    rates = plfx.gamma_rates(AIE_ALPHA, 4)
    blen = np.array([AIE_T])
    st = torch.empty(4 * 16, dtype=torch.float64, device="cuda")
    eg = torch.empty(4 * 16, dtype=torch.float64, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(blen), st, states=4, convention=plfx.PMAT_STATE)
    ctx.pmatrix(dev(e), dev(rates), dev(blen), eg, states=4, convention=plfx.PMAT_EIGEN)
    torch.cuda.synchronize()
    st = st.cpu().numpy().reshape(4, 4, 4)
    eg = eg.cpu().numpy().reshape(4, 4, 4)
    assert np.abs(st - Ps).max() < 3e-6
    ev = plfx.model_ev(e, 4, plfx.PMAT_EIGEN).reshape(4, 4)
    assert np.abs(np.einsum("ckl,ml->ckm", eg, ev) - st).max() < 1e-13


def test_device_tree_reproduces_reference_aie_golden(ctx):
    """The reference's AIE known-answer tree (four A tips, z = 0.9 on every
    branch; see tests/test_model.py) through the device path: eigen-convention
    P matrices from plfx_pmatrix, the library's EV and tip vectors, the two
    plf levels on the GPU kernels (f64) -- the cherry and the root equal the
    reference's aie/data CLVs in state coordinates to the goldens' precision."""
    import torch

    from conftest import golden
    from test_model import AIE_ALPHA, AIE_EXCH, AIE_T, aie_model

    k = golden("aie_kat.npz")
    EV_d = aie_model()[0]
    V_d = np.linalg.inv(EV_d.T)
    e = plfx.model_eigen(AIE_EXCH, EV_d[:, 0])
    V = e[4:20].reshape(4, 4)
    rates = plfx.gamma_rates(AIE_ALPHA, 4)
    P = torch.empty(64, dtype=torch.float64, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(np.array([AIE_T])), P, states=4, convention=plfx.PMAT_EIGEN)
    EV = dev(plfx.model_ev(e, 4, plfx.PMAT_EIGEN))
    tip = plfx.model_tip_vectors(e, plfx.PMAT_EIGEN).reshape(16, 4)[1]
    n = 3  # three identical sites (a ragged wave step)
    x = dev(np.tile(tip, 4 * n))
    cherry = torch.empty_like(x)
    root = torch.empty_like(x)
    ctx.plf_dev(x, x, cherry, EV, P, P)
    ctx.plf_dev(cherry, cherry, root, EV, P, P)
    torch.cuda.synchronize()
    x1 = k["x1"].astype(np.float64).reshape(4, 4)
    gold = k["golden"].astype(np.float64).reshape(4, 4)
    for got, ref in ((cherry, x1), (root, gold)):
        g = got.cpu().numpy().reshape(n, 4, 4)
        for s in range(n):
            assert np.abs(g[s] @ V.T - ref @ V_d.T).max() < 2e-6


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_traversal_with_coded_tips_reproduces_reference_aie_golden(ctx, dtype):
    """The same known-answer tree through plfx_traverse with coded tips (four
    A tips as uint8 state codes, the library's eigen-convention tip-vector
    table, one P-matrix pair per inner node from plfx_pmatrix): the root CLV
    equals the reference's golden in state coordinates (f64 to the goldens'
    six decimals, f32 to float rounding), and so does its root lnL with the
    eigen-convention root weights."""
    import torch

    from conftest import golden
    from test_model import AIE_ALPHA, AIE_EXCH, AIE_T, aie_model

    k = golden("aie_kat.npz")
    EV_d = aie_model()[0]
    V_d = np.linalg.inv(EV_d.T)
    tdt = torch.float64 if dtype == "f64" else torch.float32
    e = plfx.model_eigen(AIE_EXCH, EV_d[:, 0])
    V = e[4:20].reshape(4, 4)
    rates = plfx.gamma_rates(AIE_ALPHA, 4)
    n = 37
    # slots 0-3 tips, 4-5 cherries, 6 root; ops: [parent, child1, child2, pmat pair]
    ops = np.array([[4, 0, 1, 0], [5, 2, 3, 0], [6, 4, 5, 0]], np.int32)
    pm = torch.empty(2 * 64, dtype=tdt, device="cuda")
    ctx.pmatrix(dev(e), dev(rates), dev(np.array([AIE_T, AIE_T])), pm, states=4,
                convention=plfx.PMAT_EIGEN)
    EV = dev(plfx.model_ev(e, 4, plfx.PMAT_EIGEN)).to(tdt)
    tipvec = dev(plfx.model_tip_vectors(e, plfx.PMAT_EIGEN)).to(tdt)
    codes = torch.full((n,), 1, dtype=torch.uint8, device="cuda")  # bit 0 = A
    clv = [None] * 4 + [torch.empty(16 * n, dtype=tdt, device="cuda") for _ in range(3)]
    ctx.traverse(ops, clv, pm, EV, n, tips=[codes] * 4 + [None] * 3, tipvec=tipvec)
    torch.cuda.synchronize()
    root = clv[6].cpu().numpy().astype(np.float64).reshape(n, 4, 4)
    gold = k["golden"].astype(np.float64).reshape(4, 4)
    tol = 2e-6 if dtype == "f64" else 2e-5
    for s in range(n):
        assert np.abs(root[s] @ V.T - gold @ V_d.T).max() < tol, s
    # the root lnL with the eigen-convention root weights (w = V^T pi) equals
    # n x log of the golden's state-space likelihood, sum_c 1/4 sum_s pi_s x_s
    w = dev(plfx.model_root_weights(e, EV_d[:, 0], plfx.PMAT_EIGEN))
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    ctx.root_lnl(clv[6], n, out, catw=dev(np.full(4, 0.25)), freq=w)
    torch.cuda.synchronize()
    ref = n * np.log(np.sum(0.25 * (gold @ V_d.T) @ EV_d[:, 0]))
    assert abs(out.item() - ref) < (1e-5 if dtype == "f64" else 1e-4) * abs(ref)
