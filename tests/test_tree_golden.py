"""CPU tests: the tree-sweep oracle pinned by the reference itself.

BASELINE configs[2] (a 64-taxon post-order sweep) is, on the reference's side,
nothing but its plf() (/root/reference/app/src/plf.cpp:8-68) called once per
inner node with that node's children and P matrices.  tests/golden/tree64.npz
holds that composition as produced by the unmodified reference build
(oracle.ref_traverse over oracle/_ref; generator tests/golden/make_golden.py
make_tree64): per op the sha256 of the parent CLV, the per-site scaler bytes,
the weighted scaler sum, and the root CLV -- f32 and f64 (the reference source
with float spelled double), dense, state-coded, mixed and tip-vector tips.

Here the oracle's own sequential traversal (plf_oracle.c plfo_traverse, the
checker of every GPU traversal test) must reproduce those bytes, and the live
reference composition must too when oracle/_ref is present.  The GPU side of
the same fixture is tests/test_gpu_tree.py::test_tree64_reference_golden.
"""
import numpy as np
import pytest

from conftest import golden

CASES = [(dt, mode) for dt in (np.float32, np.float64) for mode in ("dense", "coded", "mixed", "tipvec")]


def key(dt, mode):
    return f"{'f32' if dt == np.float32 else 'f64'}_{mode}"


def check_against_golden(oracle, g, k, case, clv, sums, scal):
    ops = case["ops"]
    digests = [oracle.clv_digest(clv[int(p)]) for p in ops[:, 0]]
    bad = [j for j, (a, b) in enumerate(zip(digests, g[f"{k}_x3_sha256"])) if a != str(b)]
    assert not bad, f"{k}: parent CLVs of ops {bad[:8]} differ from the reference composition"
    assert np.array_equal(np.asarray(sums, np.int64), g[f"{k}_sums"])
    assert np.array_equal(np.stack(scal), g[f"{k}_scaler"])
    root = clv[int(ops[-1, 0])]
    assert np.array_equal(root.view(np.uint8), g[f"{k}_root"].view(np.uint8))


@pytest.mark.parametrize("dt,mode", CASES)
def test_fixture_inputs_regenerate(oracle, dt, mode):
    g = golden("tree64.npz")
    c = oracle.tree_golden_case(dt, mode, int(g["n"]), int(g["seed"]))
    assert oracle.tree_case_digest(c) == str(g[f"{key(dt, mode)}_inputs_sha256"])
    assert g[f"{key(dt, mode)}_sums"].sum() > 0  # the scaler path is in the fixture


@pytest.mark.parametrize("dt,mode", CASES)
def test_oracle_traverse_matches_reference_composition(oracle, dt, mode):
    g = golden("tree64.npz")
    c = oracle.tree_golden_case(dt, mode, int(g["n"]), int(g["seed"]))
    n, ops = c["n"], c["ops"]
    clv = [t.copy() for t in c["tips"]] + [np.zeros(16 * n, dt) for _ in range(ops.shape[0])]
    sums, scal = oracle.traverse(4, 4, ops, clv, c["pm"], c["EV"], n, c["wgt"], want_scalers=True)
    check_against_golden(oracle, g, key(dt, mode), c, clv, sums, scal)


@pytest.mark.parametrize("dt,mode", CASES)
def test_live_reference_reproduces_fixture(oracle, dt, mode):
    if not oracle.ref_available(dt):
        pytest.skip("oracle/_ref not built (no /root/reference on this machine)")
    g = golden("tree64.npz")
    c = oracle.tree_golden_case(dt, mode, int(g["n"]), int(g["seed"]))
    n, ops = c["n"], c["ops"]
    clv = [t.copy() for t in c["tips"]] + [np.zeros(16 * n, dt) for _ in range(ops.shape[0])]
    sums, scal = oracle.ref_traverse(ops, clv, c["pm"], c["EV"], n, c["wgt"], want_scalers=True)
    check_against_golden(oracle, g, key(dt, mode), c, clv, sums, scal)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_ref_scaled_sites_bisection(oracle, dt):
    """ref_scaled_sites recovers per-site scaler bytes from the reference's
    weighted sum alone: equal to the restatement's bytes on sparse, dense and
    alternating scaling."""
    if not oracle.ref_available(dt):
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(2)
    n = 999
    EV = rng.random(16).astype(dt)
    L = rng.random(64).astype(dt)
    R = rng.random(64).astype(dt)
    f = oracle._ref_call(dt)
    for pattern in (np.zeros(n, bool), np.ones(n, bool), np.arange(n) % 2 == 0, rng.random(n) < 0.01):
        x1 = rng.random(16 * n).astype(dt)
        x1.reshape(n, 16)[pattern] *= dt(1e-30) if dt == np.float64 else dt(1e-20)
        x2 = rng.random(16 * n).astype(dt)
        _, sc, _ = oracle.plf(x1, x2, EV, L, R, np.ones(n, np.int32))
        assert np.array_equal(oracle.ref_scaled_sites(f, x1, x2, EV, L, R, n), sc)


def _random_ops(rng, ntips, recycle):
    """Random topology by merging random pool members; recycle reuses consumed
    inner slots (write-after-read / write-after-write order matters)."""
    pool, free, nxt, ops = list(range(ntips)), [], ntips, []
    while len(pool) > 1:
        i, j = sorted(rng.choice(len(pool), 2, replace=False))
        a, b = pool[j], pool[i]
        pool.pop(j)
        pool.pop(i)
        if recycle and free:
            p = free.pop(0)
        else:
            p, nxt = nxt, nxt + 1
        ops.append((p, a, b, len(ops)))
        if recycle:
            free += [c for c in (a, b) if c >= ntips]
        pool.append(p)
    return np.array(ops, np.int32), nxt


@pytest.mark.parametrize("seed", range(12))
def test_random_trees_oracle_equals_reference_composition(oracle, seed):
    """Random topologies (2..40 taxa, slot recycling on odd seeds), ragged site
    counts, dense / coded / mixed tips, f32 and f64: the oracle's traversal
    (the checker of every GPU traversal test) equals the reference's plf()
    called per op, byte for byte, scaler bytes and sums included."""
    rng = np.random.default_rng(1000 + seed)
    dt = np.float32 if seed % 3 == 0 else np.float64
    if not oracle.ref_available(dt):
        pytest.skip("oracle/_ref not built")
    ntips = int(rng.integers(2, 41))
    n = int(rng.integers(1, 300))
    ops, nslots = _random_ops(rng, ntips, recycle=bool(seed % 2))
    coded = rng.random(ntips) < (0.0, 0.5, 1.0)[seed % 3]
    tips = [oracle.expand_tips(oracle.random_tip_codes(rng, n, 0.2), dt) if coded[t]
            else rng.random(16 * n).astype(dt) for t in range(ntips)]
    pm = (rng.random(ops.shape[0] * 128) * 0.3).astype(dt)
    EV = (rng.random(16) * 0.3).astype(dt)
    wgt = rng.integers(-2, 5, n).astype(np.int32)
    a = [t.copy() for t in tips] + [np.zeros(16 * n, dt) for _ in range(nslots - ntips)]
    b = [x.copy() for x in a]
    s1, sc1 = oracle.traverse(4, 4, ops, a, pm, EV, n, wgt, want_scalers=True)
    s2, sc2 = oracle.ref_traverse(ops, b, pm, EV, n, wgt, want_scalers=True)
    for s in range(nslots):
        assert np.array_equal(a[s].view(np.uint8), b[s].view(np.uint8)), s
    assert np.array_equal(s1, s2)
    for j in range(ops.shape[0]):
        assert np.array_equal(sc1[j], sc2[j]), j
