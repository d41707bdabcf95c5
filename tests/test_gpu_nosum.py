"""GPU tests of the sum-free kernel instantiations.  Every kernel is built in a
kSum form (the nodes' weighted scaler sums, reduced by block tickets) and a
sum-free form that the launchers pick when no node of a launch asks for a sum
(scaler_sum NULL -- e.g. a sweep that reads the scaler bytes, or one that
only needs the CLVs).  A kernel-trace of the GPU suite showed the sum-free
forms were never launched; here they are, through the C ABI: the CLVs and
scaler bytes must equal the oracle bit for bit (FMA mode: the oracle's fused
restatement), exactly as in the summing form."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _dna_tree(oracle, ntips, n, dtype, coded, seed):
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
@pytest.mark.parametrize("leaves", ["dense", "coded", "mixed", "left"])
@pytest.mark.parametrize("ntips,fuse", [(16, "3"), (32, "3"), (64, "3"), (64, "2"), (64, "1"), (64, "0")])
def test_dna_traverse_without_sums(oracle, dtype, leaves, ntips, fuse, monkeypatch):
    """DNA traversals with scaler bytes but no scaler sums, under every
    schedule: six-, five- and four-level passes (PLFX_FUSE=3 at 64, 32 and 16
    taxa), three-level passes (2), level pairs (1) and level batches (0);
    dense, coded, mixed or left-coded leaves (tip/tip, tip/inner and
    inner/inner nodes; left-coded: every leaf node tip/inner, so the
    three-level passes take coded leaves)."""
    import plfx
    import torch

    n = 2049
    coded = [{"dense": False, "coded": True, "mixed": t % 3 != 1, "left": t % 2 == 0}[leaves]
             for t in range(ntips)]
    ops, nslots, codes, dense, pm, EV, wgt, host = _dna_tree(oracle, ntips, n, dtype, coded, 30 + ntips)
    esums, escal = oracle.traverse(4, 4, ops, host, pm, EV, n, wgt, want_scalers=True)
    assert esums.sum() > 0
    monkeypatch.setenv("PLFX_FUSE", fuse)
    tt = torch.float64 if dtype == np.float64 else torch.float32
    c = plfx.Context(0)
    try:
        clv = [None if coded[t] else dev(dense[t]) for t in range(ntips)]
        clv += [torch.zeros(16 * n, dtype=tt, device="cuda") for _ in range(nslots - ntips)]
        tips = ([dev(codes[t]) if coded[t] else None for t in range(ntips)] + [None] * (nslots - ntips)
                if any(coded) else None)
        scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(ops.shape[0])]
        c.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, None, tips=tips)
        sched = c.last_schedule()
        torch.cuda.synchronize()
    finally:
        c.close()
    if fuse == "3" and leaves in ("dense", "coded"):
        depth = {16: "deep4", 32: "deep5", 64: "deep6"}[ntips]
        assert sched[depth] == 1, sched
    for s in range(ntips, nslots):
        assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
    for j in range(ops.shape[0]):
        assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_dna_batch_without_sums(ctx, oracle, dtype):
    """Independent DNA nodes in one batched launch, none asking for a sum."""
    import torch

    n, count = 3001, 5
    rng = np.random.default_rng(41)
    d = oracle.gen_hostmem(n, dtype, 141)
    w = rng.integers(0, 5, n).astype(np.int32)
    nodes, exp = [], []
    for i in range(count):
        x1 = (rng.random(16 * n) * (1e-12 if i % 2 == 0 else 1.0)).astype(dtype)
        x2 = rng.random(16 * n).astype(dtype)
        L, R = rng.random(64).astype(dtype), rng.random(64).astype(dtype)
        exp.append(oracle.plf(x1, x2, d["EV"], L, R, w))
        nodes.append(dict(x1=dev(x1), x2=dev(x2), x3=torch.empty(16 * n, dtype=dev(x1).dtype, device="cuda"),
                          left=dev(L), right=dev(R), scaler=torch.empty(n, dtype=torch.uint8, device="cuda")))
    ctx.plf_batch_dev(nodes, dev(d["EV"]), n, dev(w))
    torch.cuda.synchronize()
    for i, (nd, (e3, esc, _)) in enumerate(zip(nodes, exp)):
        assert np.array_equal(bits(nd["x3"].cpu().numpy()), bits(e3)), i
        assert np.array_equal(nd["scaler"].cpu().numpy(), esc), i


S, CAT = 20, 4
V = S * CAT


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("kind", ["dense", "tip1", "both"])
def test_protein_node_without_sum(ctx, oracle, dtype, fma, kind):
    """One protein node (dense, tip/dense, tip/tip) with scaler bytes and no
    sum; 2^16 + 1 sites, so every block makes several trips."""
    import torch

    n = (1 << 16) + 1
    rng = np.random.default_rng(7)
    x1 = rng.random(V * n)
    x1.reshape(n, V)[0::4] *= 1e-14
    x2 = rng.random(V * n)
    EV = rng.random(S * S) - 0.25
    L, R = rng.random(CAT * S * S), rng.random(CAT * S * S)
    if kind != "dense":
        L = L * 1e-11  # tip children: rescaled sites (a mix) through the left matrix
    w = rng.integers(0, 4, n).astype(np.int32)
    x1, x2, EV, L, R = (a.astype(dtype) for a in (x1, x2, EV, L, R))
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1 = oracle.expand_protein_tips(c1, dtype) if kind != "dense" else x1
    e2 = oracle.expand_protein_tips(c2, dtype) if kind == "both" else x2
    f3, fsc, _ = oracle.plf_generic(S, CAT, e1, e2, EV, L, R, w, fma=fma)
    assert 0 < fsc.sum() < n
    tt = torch.float64 if dtype == np.float64 else torch.float32
    x3 = torch.empty(V * n, dtype=tt, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    if kind == "dense":
        ctx.plf_dev_gen(dev(x1), dev(x2), x3, dev(EV), dev(L), dev(R), S, dev(w), sc, None, fma=fma)
    else:
        kw = dict(tip1=dev(c1))
        kw.update(tip2=dev(c2)) if kind == "both" else kw.update(x2=dev(x2))
        ctx.plf_tips_dev(x3, dev(EV), n, dev(L), dev(R), wgt=dev(w), scaler=sc, scaler_sum=None,
                         states=S, fma=fma, **kw)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
    assert np.array_equal(sc.cpu().numpy(), fsc)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("with_sum", [False, True])
def test_protein_traverse_without_sums(ctx, oracle, dtype, fma, with_sum):
    """A 16-taxon protein tree with a mix of coded and dense leaves (tip/tip,
    tip/inner and inner/inner batches), scaler bytes, with or without sums:
    every node's CLV, scaler bytes (and sum) equal a sequential evaluation by
    the oracle's generic loop in the same mode (FMA included, f32 too)."""
    import torch

    n, ntips = 700, 16
    rng = np.random.default_rng(16)
    ops = oracle.balanced_tree_ops(ntips)
    nops, nslots = ops.shape[0], ntips + ops.shape[0]
    coded = [t % 3 != 2 for t in range(ntips)]
    codes = [oracle.random_protein_codes(rng, n, 0.2) for _ in range(ntips)]
    dense = [rng.random(V * n).astype(dtype) for _ in range(ntips)]
    pm = (rng.random(nops * 2 * CAT * S * S) * 0.05).astype(dtype)
    EV = (rng.random(S * S) * 0.05).astype(dtype)
    wgt = rng.integers(1, 4, n).astype(np.int32)
    host = [oracle.expand_protein_tips(codes[t], dtype) if coded[t] else dense[t].copy()
            for t in range(ntips)] + [None] * nops
    escal, einc = [], []
    M = CAT * S * S
    for parent, a, b, p in ops:  # post order: children before parents
        x3, sc, inc = oracle.plf_generic(S, CAT, host[a], host[b], EV, pm[2 * p * M:(2 * p + 1) * M],
                                         pm[(2 * p + 1) * M:(2 * p + 2) * M], wgt, fma=fma)
        host[parent] = x3
        escal.append(sc)
        einc.append(inc)
    assert sum(einc) > 0
    tt = torch.float64 if dtype == np.float64 else torch.float32
    clv = [None if coded[t] else dev(dense[t]) for t in range(ntips)]
    clv += [torch.zeros(V * n, dtype=tt, device="cuda") for _ in range(nops)]
    tips = [dev(codes[t]) if coded[t] else None for t in range(ntips)] + [None] * nops
    scal = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(nops)]
    sums = torch.full((nops,), -1, dtype=torch.int64, device="cuda") if with_sum else None
    ctx.traverse(ops, clv, dev(pm), dev(EV), n, dev(wgt), scal, sums, tips=tips, states=S, fma=fma)
    torch.cuda.synchronize()
    for s in range(ntips, nslots):
        assert np.array_equal(bits(clv[s].cpu().numpy()), bits(host[s])), s
    for j in range(nops):
        assert np.array_equal(scal[j].cpu().numpy(), escal[j]), j
    if with_sum:
        assert sums.cpu().tolist() == einc


@pytest.mark.parametrize("kind", ["dense", "tip1"])
def test_protein_fma_queue_without_sum(ctx, oracle, kind):
    """The f64 FMA protein kernel's device-wide tile queue (from 32 tiles per
    block: 2^20 sites) without a sum, dense and tip/dense: windows at the
    start, middle and end checked bit for bit against the oracle's fused
    restatement on those sites (sites are independent)."""
    import torch

    n = (1 << 20) + 37
    rng = np.random.default_rng(20)
    x1 = rng.random(V * n)
    x1.reshape(n, V)[0::4] *= 1e-14
    x2 = rng.random(V * n)
    EV = rng.random(S * S) - 0.25
    L, R = rng.random(CAT * S * S), rng.random(CAT * S * S)
    if kind == "tip1":
        L = L * 1e-11
    w = rng.integers(0, 4, n).astype(np.int32)
    c1 = oracle.random_protein_codes(rng, n, 0.3)
    x3 = torch.empty(V * n, dtype=torch.float64, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    if kind == "dense":
        ctx.plf_dev_gen(dev(x1), dev(x2), x3, dev(EV), dev(L), dev(R), S, dev(w), sc, None, fma=True)
    else:
        ctx.plf_tips_dev(x3, dev(EV), n, dev(L), dev(R), tip1=dev(c1), x2=dev(x2), wgt=dev(w), scaler=sc,
                         scaler_sum=None, states=S, fma=True)
    torch.cuda.synchronize()
    g3, gsc = x3.cpu().numpy(), sc.cpu().numpy()
    for lo in (0, n // 2 - 2048, n - 4096):
        win = slice(lo, lo + 4096)
        e1 = oracle.expand_protein_tips(c1[win]) if kind == "tip1" else x1[V * lo:V * (lo + 4096)]
        f3, fsc, _ = oracle.plf_generic(S, CAT, e1, x2[V * lo:V * (lo + 4096)], EV, L, R, w[win], fma=True)
        assert np.array_equal(bits(g3[V * lo:V * (lo + 4096)]), bits(f3)), lo
        assert np.array_equal(gsc[win], fsc), lo
    assert 0 < int(gsc.sum()) < n
