"""CPU tests: pin the oracle (oracle/plf_oracle.c, oracle/oracle.py) before it
is trusted as the checker of the GPU path.

Pins, in order of strength:
  * the reference's own AIE golden vectors (aie/data/golden{0..3}.txt), parsed
    into tests/golden/aie_kat.npz;
  * fixtures produced by the unmodified reference plf() (tests/golden/
    hostmem_f32_*.npz/json, edge_f32.npz; generator tests/golden/make_golden.py);
  * the reference plf() itself, live, when oracle/_ref was built;
  * std::mt19937 draws (tests/golden/mt19937.npz) for the input generator;
  * the AIE PLIO stimulus files (aie/data/inputcombinedev*, stream/*) for the
    restated mm2s movers and the instance packing.
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, golden


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def test_mt19937_matches_std(oracle):
    g = golden("mt19937.npz")
    raw, dbl = oracle.mt_draws(int(g["seed"]), 2000)
    assert np.array_equal(raw, g["raw"])
    assert np.array_equal(dbl[:1000].view(np.uint64), g["canonical"].view(np.uint64))


def test_aie_kat_golden(oracle):
    """plf() restatement reproduces aie/data/golden{0..3}.txt exactly."""
    k = golden("aie_kat.npz")
    x3, sc, inc = oracle.plf(k["x1"], k["x2"], k["EV"], k["left"], k["right"], np.ones(1, np.int32))
    g = k["golden"]
    nz = g != 0
    assert np.array_equal(x3[nz], g[nz])           # 0 relative error on nonzero entries
    assert np.all(np.abs(x3[~nz]) <= 1e-6)          # golden 0.0 entries (cancellation)
    assert sc[0] == 0 and inc == 0
    # independent numpy cross-check of the AIE lane formula ((x.B_L)*(y.B_R)).EV
    for c in range(4):
        BL = k["left"][c * 16:(c + 1) * 16].reshape(4, 4).T
        BR = k["right"][c * 16:(c + 1) * 16].reshape(4, 4).T
        ref = oracle.aie_lane_compute(k["x1"][4 * c:4 * c + 4], k["x2"][4 * c:4 * c + 4], BL, BR,
                                      k["EV"].reshape(4, 4))
        assert np.allclose(ref, g[4 * c:4 * c + 4], rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("n", [1024, 1000])
def test_hostmem_fixture_inputs_regenerate(oracle, n):
    g = golden(f"hostmem_f32_n{n}.npz")
    d = oracle.gen_hostmem(n, np.float32, int(g["seed"]))
    for key in ("EV", "left", "right", "x1", "x2", "wgt"):
        assert np.array_equal(bits(d[key]) if d[key].dtype != np.int32 else d[key],
                              bits(g[key]) if g[key].dtype != np.int32 else g[key]), key


@pytest.mark.parametrize("n", [1024, 1000, 4096])
def test_hostmem_fixture_bitexact(oracle, n):
    g = golden(f"hostmem_f32_n{n}.npz")
    d = oracle.gen_hostmem(n, np.float32, int(g["seed"]))
    x3, sc, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    assert np.array_equal(bits(x3), bits(g["x3"]))
    assert np.array_equal(sc, g["scaler"])
    assert inc == int(g["scalerIncrement"]) == n // 4 + (n % 4 > 0)  # every 4th site scales


def test_hostmem_65536_hash(oracle):
    rec = json.loads((GOLDEN / "hostmem_f32_n65536.json").read_text())
    d = oracle.gen_hostmem(rec["n"], np.float32, rec["seed"])
    x3, sc, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    assert hashlib.sha256(x3.tobytes()).hexdigest() == rec["x3_sha256"]
    assert inc == rec["scalerIncrement"] == rec["n"] // 4


def test_edge_sites(oracle):
    """Boundary semantics: strict < 2^-32, |x|, NaN/inf never scale, zeros and
    denormals scale, ragged weights."""
    g = golden("edge_f32.npz")
    x3, sc, inc = oracle.plf(g["x1"], g["x2"], g["EV"], g["left"], g["right"], g["wgt"])
    assert np.array_equal(bits(x3), bits(g["x3"]))
    assert np.array_equal(sc, g["scaler"])
    assert inc == int(g["scalerIncrement"])
    assert list(sc) == [1, 0, 0, 1, 1, 1, 0, 0, 1, 0, 0, 1]


def test_reference_binary_live(oracle):
    """Restatement == the reference plf() built from /root/reference (when
    oracle/_ref exists; it travels with the snapshot)."""
    if oracle.ref_lib("O0") is None:
        pytest.skip("oracle/_ref not built")
    for n, seed in ((777, 1), (2048, 99)):
        d = oracle.gen_hostmem(n, np.float32, seed)
        w = (np.arange(n) % 5 + 1).astype(np.int32)
        x3, sc, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w)
        for opt in ("O0", "O3"):
            r3, rinc = oracle.ref_plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w, opt)
            assert np.array_equal(bits(x3), bits(r3)), opt
            assert inc == rinc


def test_reference_double_instantiation_live(oracle):
    """Pins the f64 restatement: the reference's own plf() loop compiled in
    double (oracle/ref_shim_f64.cpp builds the unmodified plf.cpp with float
    spelled double) equals the oracle's f64 plf() bit for bit, at -O0 and -O3,
    on host_mem-protocol inputs, on inputs where every 4th site underflows,
    and on hand-built edge sites (values straddling 2^-32, signed zeros)."""
    if oracle.ref_lib_f64("O0") is None:
        pytest.skip("oracle/_ref has no f64 build")
    rng = np.random.default_rng(5)
    cases = []
    for n, seed in ((777, 1), (4096, 99)):
        d = oracle.gen_hostmem(n, np.float64, seed)
        cases.append((d, (np.arange(n) % 5 + 1).astype(np.int32)))
    d = oracle.gen_hostmem(1024, np.float64, 3)
    d["x1"].reshape(-1, 16)[::4] *= 1e-30
    d["x2"].reshape(-1, 16)[1::4] *= -1e-25
    cases.append((d, d["wgt"]))
    e = oracle.gen_hostmem(64, np.float64, 11)
    e["x1"].reshape(-1, 16)[:, :] = rng.choice([0.0, -0.0, 2.0 ** -33, 2.0 ** -32, 1e-300, 1.0],
                                              size=(64, 16))
    cases.append((e, e["wgt"]))
    for d, w in cases:
        x3, sc, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w)
        assert sc.any() or d["x1"].size != 16 * 1024
        for opt in ("O0", "O3"):
            r3, rinc = oracle.ref_plf_f64(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w, opt)
            assert np.array_equal(bits(x3), bits(r3)), opt
            assert inc == rinc


def test_double_and_generic_agree(oracle):
    d = oracle.gen_hostmem(513, np.float64, 7)
    x3, sc, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    g3, gsc, ginc = oracle.plf_generic(4, 4, d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    assert np.array_equal(bits(x3), bits(g3)) and np.array_equal(sc, gsc) and inc == ginc
    o3, osc, oinc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"], threads=4)
    assert np.array_equal(bits(x3), bits(o3)) and np.array_equal(sc, osc) and inc == oinc
    # the f64 result is the f32 computation up to rounding
    f = oracle.gen_hostmem(513, np.float32, 7)
    f3, fsc, finc = oracle.plf(f["x1"], f["x2"], f["EV"], f["left"], f["right"], f["wgt"])
    assert np.array_equal(fsc, sc)
    assert np.allclose(f3, x3, rtol=1e-5, atol=0)


def test_scaler_sum(oracle):
    sc = (np.arange(1000) % 3 == 0).astype(np.uint8)
    w = (np.arange(1000) % 7).astype(np.int32)
    assert oracle.scaler_sum(sc, w) == int((sc.astype(np.int64) * w).sum())
    assert oracle.scaler_sum(sc) == int(sc.sum())


def test_mover_emulation_matches_aie_stimuli(oracle):
    """mm2sleft/mm2sright (Comb, window 16288 B = 1018 sites) and the stream
    variant reproduce the reference's AIE PLIO stimulus files beat for beat,
    which pins the instance packing (host_mem.cpp:221-243) and the P transpose."""
    k = golden("aie_kat.npz")
    n = 1018
    x1 = np.tile(k["x1"], n)
    x2 = np.tile(k["x2"], n)
    tb = oracle.Testbench(n, 1, 16288, oracle.COMBINED)
    L, R = oracle.pack_instance(tb, 0, k["EV"], k["left"], k["right"], x1, x2)
    ls = oracle.mm2s_lane_streams(L, n, 16288, "left", oracle.COMBINED)
    rs = oracle.mm2s_lane_streams(R, n, 16288, "right", oracle.COMBINED)
    for c in range(4):
        assert np.array_equal(ls[c], k[f"combinedevleft{c}"])
        assert np.array_equal(rs[c], k[f"combinedevright{c}"])
    tbs = oracle.Testbench(64, 1, 1024, oracle.COMBINED, oracle.STREAM)
    L, R = oracle.pack_instance(tbs, 0, k["EV"], k["left"], k["right"], np.tile(k["x1"], 64),
                                np.tile(k["x2"], 64))
    ls = oracle.mm2s_lane_streams(L, 64, 0, "left", oracle.COMBINED, aie="stream")
    rs = oracle.mm2s_lane_streams(R, 64, 0, "right", oracle.COMBINED, aie="stream")
    for c in range(4):
        assert np.array_equal(ls[c], k[f"stream_combinedevleft{c}"])
        assert np.array_equal(rs[c], k[f"stream_combinedevright{c}"])


def test_sw_emu_plumbing_1024(oracle):
    """BASELINE config #1: the sw_emu-style CPU path -- pack per instance,
    stream through the restated movers and AIE lane arithmetic, s2mm rescale --
    equals the reference plf() on 1024 sites (window PLIO, 1 inner node)."""
    g = golden("hostmem_f32_n1024.npz")
    n = 1024
    for layout, P, W in ((oracle.SEPARATE, 1, 8192), (oracle.COMBINED, 3, 1024), (oracle.SEPARATE, 4, 16288)):
        tb = oracle.Testbench(n, P, W, layout)
        out = np.empty(n * 16, np.float32)
        scal = np.empty(n, np.uint8)
        for kk in range(P):
            nk = tb.alignments_per_instance(kk)
            off = tb.instance_site_offset(kk)
            L, R = oracle.pack_instance(tb, kk, g["EV"], g["left"], g["right"], g["x1"], g["x2"])
            ls = oracle.mm2s_lane_streams(L, nk, W, "left", layout)
            rs = oracle.mm2s_lane_streams(R, nk, W, "right", layout)
            if layout == oracle.SEPARATE:
                ldata, rdata = ls["data"], rs["data"]
                hdr = 0
            else:
                ldata, rdata = ls, rs
                hdr = 6
            apw = W >> 4
            lane_out = []
            for c in range(4):
                # per window: header beats then apw site beats; run the lane
                # math in float32 through the restated plf() one category at a time
                xs_l = np.concatenate([ldata[c][w * (apw + hdr) + hdr:(w + 1) * (apw + hdr)]
                                       for w in range(tb.num_windows_per_instance())])
                xs_r = np.concatenate([rdata[c][w * (apw + hdr) + hdr:(w + 1) * (apw + hdr)]
                                       for w in range(tb.num_windows_per_instance())])
                lane_out.append((xs_l, xs_r))
            # reassemble sites and evaluate with the oracle (the lane arithmetic)
            slots = lane_out[0][0].shape[0]
            xl = np.stack([lane_out[c][0] for c in range(4)], axis=1).reshape(slots * 16)
            xr = np.stack([lane_out[c][1] for c in range(4)], axis=1).reshape(slots * 16)
            x3, _, _ = oracle.plf(np.ascontiguousarray(xl), np.ascontiguousarray(xr), g["EV"],
                                  g["left"], g["right"])
            # undo plf()'s own rescale, let s2mm do it with the padding mask
            raw3, sraw, _ = oracle.plf(np.ascontiguousarray(xl), np.ascontiguousarray(xr), g["EV"],
                                       g["left"], g["right"])
            unscaled = raw3.reshape(slots, 16).copy()
            unscaled[sraw == 1] = (unscaled[sraw == 1].astype(np.float64) / oracle.TWO_TO_32).astype(np.float32)
            lanes = [unscaled[:, 4 * c:4 * c + 4] for c in range(4)]
            mem, sc = oracle.s2mm(lanes, nk, W)
            out[off * 16:(off + nk) * 16] = mem[:nk * 16]
            scal[off:off + nk] = sc[:nk]
        assert np.array_equal(bits(out), bits(g["x3"])), (layout, P, W)
        assert np.array_equal(scal, g["scaler"])
        assert int(scal.astype(np.int64).sum()) == int(g["scalerIncrement"])


@pytest.mark.parametrize("N,P,W,layout,aie", [
    (1024, 1, 8192, 1, 1), (1000000, 9, 8192, 1, 1), (1000, 3, 1024, 0, 1),
    (12345, 4, 16288, 0, 1), (999, 2, 1024, 1, 0), (7, 1, 16384, 0, 1),
])
def test_testbench_sizing_examples(oracle, N, P, W, layout, aie):
    tb = oracle.Testbench(N, P, W, layout, aie)
    total = sum(tb.alignments_per_instance(k) for k in range(P))
    assert total == N
    assert tb.instance_site_offset(P - 1) + tb.alignments_per_instance(P - 1) == N
    if aie == 1:
        assert tb.elements_per_instance() % (W >> 4 << 4) == 0
        assert tb.elements_per_instance() >= tb.alignments_per_instance() * 16
    # 1M sites, W=8192 -> 1954 windows -> 1,000,448 padded sites
    if (N, P, W) == (1000000, 9, 8192):
        assert tb.alignments_per_instance() == 111112


def test_tip_expansion_definition(oracle):
    """Tip codes (plfx.h section 8): bit s -> state s, every category, upper
    nibble ignored."""
    codes = np.array([0, 1, 2, 4, 8, 5, 15, 0xF1, 0x30], np.uint8)
    x = oracle.expand_tips(codes).reshape(-1, 4, 4)
    exp = np.array([[0, 0, 0, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1],
                    [1, 0, 1, 0], [1, 1, 1, 1], [1, 0, 0, 0], [0, 0, 0, 0]], np.float64)
    for c in range(4):
        assert np.array_equal(x[:, c, :], exp)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_tip_table_identity(oracle, dtype):
    """The GPU tip path reads ump[k] = T[c][code][k] = sum_l bit_l * P_c[k][l]
    (ascending l from +0.0) from a per-block table.  Restated here in numpy
    with the same operation order, the per-site result must equal plf() on the
    expanded CLV bit for bit -- the algebraic claim the kernel relies on."""
    rng = np.random.default_rng(11)
    n = 3000
    c1 = oracle.random_tip_codes(rng, n, 0.3)
    c2 = oracle.random_tip_codes(rng, n, 0.3)
    L = rng.random(64).astype(dtype)
    R = rng.random(64).astype(dtype)
    EV = rng.random(16).astype(dtype)
    x3, sc, inc = oracle.plf(oracle.expand_tips(c1, dtype), oracle.expand_tips(c2, dtype), EV, L, R)

    def table(P):
        t = np.zeros((4, 16, 4), dtype)
        for code in range(16):
            for l in range(4):
                t[:, code, :] += dtype((code >> l) & 1) * P.reshape(4, 4, 4)[:, :, l]
        return t

    u1 = table(L)[:, c1 & 15, :].transpose(1, 0, 2)   # (n, c, k)
    u2 = table(R)[:, c2 & 15, :].transpose(1, 0, 2)
    p = u1 * u2
    o = np.zeros((n, 4, 4), dtype)
    E = EV.reshape(4, 4)
    for k in range(4):
        o += p[:, :, k:k + 1] * E[k][None, None, :]
    small = np.all(np.abs(o.reshape(n, 16)) < dtype(2.0 ** -32), axis=1)
    o[small] *= dtype(2.0 ** 32)
    assert np.array_equal(bits(o.reshape(-1)), bits(x3))
    assert np.array_equal(sc, small.astype(np.uint8))
    assert int(inc) == int(small.sum())


def test_protein_tip_expansion():
    """The protein tip table (plfx.h section 8): one-hot rows, B = N|D,
    Z = Q|E, X and gap all ones, codes >= 24 read row 23."""
    import numpy as np

    import oracle as O

    t = O.protein_tip_table()
    assert t.shape == (24, 20) and (t[:20] == np.eye(20)).all()
    assert list(np.flatnonzero(t[20])) == [2, 3] and list(np.flatnonzero(t[21])) == [5, 6]
    assert (t[22:] == 1).all()
    x = O.expand_protein_tips(np.array([3, 20, 200], np.uint8))
    assert x.shape == (3 * 80,)
    r = x.reshape(3, 4, 20)
    assert (r[:, 0] == r[:, 3]).all() and r[0, 0, 3] == 1 and r[0, 0].sum() == 1
    assert r[1, 2].sum() == 2 and (r[2] == 1).all()


def _adversarial_inputs(n, dtype, seed):
    """CLVs and matrices built to hit the sign of zero: many +-0.0 entries,
    negative matrix entries and zeros, products that underflow."""
    rng = np.random.default_rng(seed)
    tiny = np.finfo(dtype).tiny

    def field(size, neg):
        v = rng.random(size).astype(dtype)
        if neg:
            v = v - dtype(0.5)
        r = rng.random(size)
        v[r < 0.3] = dtype(0.0)
        v[(r >= 0.3) & (r < 0.5)] = dtype(-0.0)
        v[(r >= 0.5) & (r < 0.55)] *= tiny  # products underflow to +-0
        return v

    return (field(16 * n, True), field(16 * n, True), field(16, True),
            field(64, True), field(64, True))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_ump_chain_start_is_exact(oracle, dtype):
    """The kernels start each ump chain at its first product instead of +0.0
    (plf_dna.hpp, site_cat).  Proof by exhaustion over adversarial inputs:
    numpy restatement of both chain forms, element-wise in plf()'s order, gives
    bit-identical x3 -- and both equal the C oracle."""
    n = 20000
    x1, x2, EV, left, right = _adversarial_inputs(n, dtype, 7)
    a = x1.reshape(n, 4, 4)
    b = x2.reshape(n, 4, 4)
    PL = left.reshape(4, 4, 4)
    PR = right.reshape(4, 4, 4)
    E = EV.reshape(4, 4)
    z = dtype(0.0)
    out = {}
    for form in ("zero", "first"):
        p = np.empty((n, 4, 4), dtype)
        for k in range(4):
            u1 = (z + a[:, :, 0] * PL[None, :, k, 0]) if form == "zero" else a[:, :, 0] * PL[None, :, k, 0]
            u2 = (z + b[:, :, 0] * PR[None, :, k, 0]) if form == "zero" else b[:, :, 0] * PR[None, :, k, 0]
            for l in range(1, 4):
                u1 = u1 + a[:, :, l] * PL[None, :, k, l]
                u2 = u2 + b[:, :, l] * PR[None, :, k, l]
            p[:, :, k] = u1 * u2
        x3 = np.empty((n, 4, 4), dtype)
        for l in range(4):
            o = np.full((n, 4), z)
            for k in range(4):
                o = o + p[:, :, k] * E[k, l]
            x3[:, :, l] = o
        out[form] = x3.reshape(-1)
    assert np.array_equal(bits(out["zero"]), bits(out["first"]))
    # the first products include -0.0, where 0 + q0 and q0 differ: the test bites
    q0 = a[:, :, 0] * PL[None, :, 0, 0]
    assert np.any((q0 == 0) & np.signbit(q0))
    e3, _, _ = oracle.plf(x1, x2, EV, left, right)
    small = np.abs(out["zero"]).reshape(n, 16).max(axis=1) < (2.0 ** -32)
    exp = out["zero"].reshape(n, 16).copy()
    exp[small] *= dtype(2.0 ** 32)
    assert np.array_equal(bits(exp.reshape(-1)), bits(e3))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("fma", [False, True])
def test_generic_openmp_equals_serial(dtype, fma):
    """The OpenMP generic loop (the protein CPU baseline) gives the serial
    loop's x3, scaler bytes and weighted sum at ragged thread splits."""
    import oracle as O

    rng = np.random.default_rng(3)
    S, Cc = 20, 4
    for n in (1, 7, 1001):
        x1 = rng.random(S * Cc * n).astype(dtype)
        x1.reshape(n, -1)[0::3] *= 1e-14
        x2 = rng.random(S * Cc * n).astype(dtype)
        EV = (rng.random(S * S) - 0.25).astype(dtype)
        L, R = (rng.random(Cc * S * S).astype(dtype) for _ in range(2))
        w = rng.integers(0, 4, n).astype(np.int32)
        ser = O.plf_generic(S, Cc, x1, x2, EV, L, R, w, fma=fma)
        for threads in (1, 3, 8):
            par = O.plf_generic(S, Cc, x1, x2, EV, L, R, w, fma=fma, threads=threads)
            assert np.array_equal(ser[0], par[0]) and np.array_equal(ser[1], par[1])
            assert ser[2] == par[2]


@pytest.mark.parametrize("S", [4, 20])
def test_generic_against_independent_numpy(oracle, S):
    """The generic S-state restatement (the protein oracle, an unpinned
    extension of the pinned loop) against an independent numpy statement of
    the same mathematics: U = P_L x1, V = P_R x2 per category, x3 = EV^T (U * V),
    rescaled by 2^32 where every value of the site is below 2^-32.  Different
    summation order, so within 1e-13 relative (positive inputs: no
    cancellation); identical scaler decisions and weighted sum."""
    rng = np.random.default_rng(20 + S)
    Cc, n = 4, 777
    x1 = rng.random((n, Cc, S))
    x1[0::5] *= 1e-14                      # clearly rescaled sites
    x2 = rng.random((n, Cc, S))
    P_L, P_R = rng.random((Cc, S, S)), rng.random((Cc, S, S))
    EV = rng.random((S, S))
    w = rng.integers(0, 5, n).astype(np.int32)
    g3, gsc, ginc = oracle.plf_generic(S, Cc, x1.ravel(), x2.ravel(), EV.ravel(), P_L.ravel(),
                                       P_R.ravel(), w)
    U = np.einsum("ckl,icl->ick", P_L, x1)
    Vv = np.einsum("ckl,icl->ick", P_R, x2)
    x3 = np.einsum("ick,kl->icl", U * Vv, EV)
    sc = np.all(np.abs(x3.reshape(n, -1)) < 2.0 ** -32, axis=1)
    x3[sc] *= 2.0 ** 32
    assert np.array_equal(gsc.astype(bool), sc) and sc.sum() >= n // 5
    assert ginc == int((sc * w).sum())
    assert np.allclose(g3, x3.ravel(), rtol=1e-13, atol=0)
