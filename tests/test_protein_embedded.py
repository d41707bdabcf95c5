"""CPU tests: the S-state (protein) restatement pinned by the reference on the
embedded 4-state sub-space.

The reference's plf() (/root/reference/app/src/plf.cpp:8-68) is hard-wired to 4
states, so a 20-state node has no reference output in general.  But a DNA
problem embedded in the first 4 of 20 states (CLV states 4..19 = +0.0, P and
EV zero outside their top-left 4x4 block; oracle.embed_dna_*) makes plf()'s
20-state loop add only exact +0.0 terms to the 4-state chains and test only
extra +0.0 values in the scale check, so states 0..3 of the 20-state result
must equal the reference's 4-state plf() bit for bit and states 4..19 must
stay +0.0 (exact mode, f32 and f64).  Here the oracle's generic S-state loop
(plfo_plf_gen_*, the checker of every protein GPU test) and its S-state
traversal are held to that, against the live reference build and against
tests/golden/tree64.npz; tests/test_gpu_protein.py::test_protein_embedded_dna_*
hold the GPU's protein kernels to the same.
"""
import numpy as np
import pytest

from conftest import golden

S = 20


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("n", [1, 63, 1000])
def test_generic_loop_on_embedded_dna_equals_reference(oracle, dt, n):
    if not oracle.ref_available(dt):
        pytest.skip("oracle/_ref not built")
    d = oracle.gen_hostmem(n, dt, 77 + n)
    w = np.arange(n, dtype=np.int32) % 5 - 1
    f = oracle._ref_call(dt)
    r3 = np.empty(16 * n, dt)
    rinc = f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w)
    rsc = oracle.ref_scaled_sites(f, d["x1"], d["x2"], d["EV"], d["left"], d["right"], n)
    x3, sc, inc = oracle.plf_generic(S, 4, oracle.embed_dna_clv(d["x1"]), oracle.embed_dna_clv(d["x2"]),
                                     oracle.embed_dna_mats(d["EV"]), oracle.embed_dna_mats(d["left"]),
                                     oracle.embed_dna_mats(d["right"]), w)
    got, rest_zero = oracle.extract_dna_clv(x3)
    assert rest_zero
    assert np.array_equal(got.view(np.uint8), r3.view(np.uint8))
    assert np.array_equal(sc, rsc) and inc == rinc
    assert rsc.sum() > 0 or n < 4


def embedded_tree(oracle, g, dt, mode):
    """The tree64 golden case in 20 states: (case, ops, dense protein tips,
    protein codes per tip (None for dense), protein P pairs, EV)."""
    c = oracle.tree_golden_case(dt, mode, int(g["n"]), int(g["seed"]))
    tips = [oracle.embed_dna_clv(t) for t in c["tips"]]
    codes = [None if cd is None else (cd & 15).astype(np.uint8) for cd in c["codes"]]
    return c, tips, codes, oracle.embed_dna_mats(c["pm"]), oracle.embed_dna_mats(c["EV"])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("mode", ["dense", "coded", "mixed"])
def test_generic_traversal_on_embedded_tree_equals_golden(oracle, dt, mode):
    g = golden("tree64.npz")
    k = f"{'f32' if dt == np.float32 else 'f64'}_{mode}"
    c, tips, codes, pm, EV = embedded_tree(oracle, g, dt, mode)
    n, ops = c["n"], c["ops"]
    # coded tips as the protein kernels read them: rows of the embedded table
    tv = oracle.embedded_dna_tipvec(dt).reshape(oracle.PROT_CODES, S)
    for t, cd in enumerate(codes):
        if cd is not None:
            rows = tv[np.minimum(cd, oracle.PROT_CODES - 1)]
            assert np.array_equal(np.repeat(rows[:, None, :], 4, axis=1).reshape(-1), tips[t])
    clv = [t.copy() for t in tips] + [np.zeros(4 * S * n, dt) for _ in range(ops.shape[0])]
    sums, scal = oracle.traverse(S, 4, ops, clv, pm, EV, n, c["wgt"], want_scalers=True)
    digests = []
    for p in ops[:, 0]:
        x, rest_zero = oracle.extract_dna_clv(clv[int(p)])
        assert rest_zero
        digests.append(oracle.clv_digest(x))
    bad = [j for j, (a, b) in enumerate(zip(digests, g[f"{k}_x3_sha256"])) if a != str(b)]
    assert not bad, bad[:8]
    assert np.array_equal(sums, g[f"{k}_sums"])
    assert np.array_equal(np.stack(scal), g[f"{k}_scaler"])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("seed", range(6))
def test_fma_restatement_equals_contracted_reference(oracle, dt, seed):
    """PLFX_FMA's semantics -- plf()'s loop with every multiply-add fused, in
    plf()'s order -- pinned by the reference source itself compiled with FMA
    contraction (oracle/_ref/libplfref{,_f64}_fma.so): the oracle's fma
    restatement at S = 4 equals it bit for bit (and differs from the unfused
    build, so the test sees the fusion)."""
    if not oracle.ref_available(dt, "fma"):
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 4000))
    d = oracle.gen_hostmem(n, dt, 300 + seed)
    x1 = d["x1"] if seed % 2 else ((rng.random(16 * n) - 0.5) * 1e-9).astype(dt)  # signed, scaling
    w = rng.integers(-3, 5, n).astype(np.int32)
    f = oracle._ref_call(dt, "fma")
    r3 = np.empty(16 * n, dt)
    rinc = f(x1, d["x2"], r3, d["EV"], n, d["left"], d["right"], w)
    e3, esc, einc = oracle.plf_generic(4, 4, x1, d["x2"], d["EV"], d["left"], d["right"], w, fma=True)
    assert np.array_equal(e3.view(np.uint8), r3.view(np.uint8)) and einc == rinc
    assert np.array_equal(esc, oracle.ref_scaled_sites(f, x1, d["x2"], d["EV"], d["left"], d["right"], n))
    u3, _, _ = oracle.plf(x1, d["x2"], d["EV"], d["left"], d["right"], w)
    assert not np.array_equal(u3.view(np.uint8), r3.view(np.uint8))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_generic_fma_loop_on_embedded_dna_equals_contracted_reference(oracle, dt):
    """The S = 20 fma restatement (the checker of the protein FMA kernels) on
    the embedded sub-space equals the FMA-contracted reference on the 4-state
    problem: the extra terms are fma(0, 0, v) = v exactly."""
    if not oracle.ref_available(dt, "fma"):
        pytest.skip("oracle/_ref not built")
    n = 2049
    d = oracle.gen_hostmem(n, dt, 808)
    w = (np.arange(n, dtype=np.int32) % 4)
    f = oracle._ref_call(dt, "fma")
    r3 = np.empty(16 * n, dt)
    rinc = f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w)
    x3, sc, inc = oracle.plf_generic(S, 4, oracle.embed_dna_clv(d["x1"]), oracle.embed_dna_clv(d["x2"]),
                                     oracle.embed_dna_mats(d["EV"]), oracle.embed_dna_mats(d["left"]),
                                     oracle.embed_dna_mats(d["right"]), w, fma=True)
    got, rest_zero = oracle.extract_dna_clv(x3)
    assert rest_zero and np.array_equal(got.view(np.uint8), r3.view(np.uint8)) and inc == rinc


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("fma", [False, True])
def test_generic_loop_on_five_dna_blocks_equals_reference(oracle, dt, fma):
    """Five 4-state problems side by side (states 4b..4b+3, block-diagonal P
    and EV) cover every state position of the 20-state loop: each block
    equals its own reference plf() (exact: the reference build; FMA: the
    contracted build), given the blocks share the scaling pattern (the
    host_mem protocol scales every 4th site in each)."""
    opt = "fma" if fma else "O0"
    if not oracle.ref_available(dt, opt):
        pytest.skip("oracle/_ref not built")
    n = 1001
    ps = [oracle.gen_hostmem(n, dt, 900 + b) for b in range(5)]
    w = np.arange(n, dtype=np.int32) % 3
    f = oracle._ref_call(dt, opt)
    refs, incs = [], []
    for d in ps:
        r3 = np.empty(16 * n, dt)
        incs.append(f(d["x1"], d["x2"], r3, d["EV"], n, d["left"], d["right"], w))
        refs.append(r3)
    x3, sc, inc = oracle.plf_generic(S, 4, oracle.embed_clv_blocks([d["x1"] for d in ps]),
                                     oracle.embed_clv_blocks([d["x2"] for d in ps]),
                                     oracle.embed_mat_blocks([d["EV"] for d in ps]),
                                     oracle.embed_mat_blocks([d["left"] for d in ps]),
                                     oracle.embed_mat_blocks([d["right"] for d in ps]), w, fma=fma)
    outs, rest_zero = oracle.extract_clv_blocks(x3, 5)
    assert rest_zero
    for b in range(5):
        assert np.array_equal(outs[b].view(np.uint8), refs[b].view(np.uint8)), b
    assert len(set(incs)) == 1 and inc == incs[0]
