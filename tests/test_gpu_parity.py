"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
reference-produced fixtures.  Bar: bit-exact scaler bytes/sums and bit-exact
CLVs in f32 (the reference's exact-equality check, host_mem.cpp:421-439); in
f64 bit-exact against the oracle's double instantiation, and in any case
within the north-star tolerance |a-b| <= 1e-10 * |b| (asserted separately)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, golden, check_report_rows

pytestmark = pytest.mark.gpu

F64_RTOL = 1e-10  # BASELINE.json north_star: fp64 CLVs within 1e-10 relative


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def torch_dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def rel_ok(got, exp):
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    fin = np.isfinite(exp)
    assert np.array_equal(np.isnan(got), np.isnan(exp))
    assert np.all(np.abs(got[fin] - exp[fin]) <= F64_RTOL * np.abs(exp[fin]))


@pytest.mark.parametrize("n", [1024, 1000, 4096])
def test_plf_f32_reference_fixtures(ctx, oracle, n):
    g = golden(f"hostmem_f32_n{n}.npz")
    d = oracle.gen_hostmem(n, np.float32, int(g["seed"]))
    x3 = np.zeros(16 * n, np.float32)
    inc = ctx.plf(d["x1"], d["x2"], x3, d["EV"], n, d["left"], d["right"], d["wgt"])
    assert np.array_equal(bits(x3), bits(g["x3"]))
    assert inc == int(g["scalerIncrement"])


def test_plf_f32_65536_hash(ctx, oracle):
    rec = json.loads((GOLDEN / "hostmem_f32_n65536.json").read_text())
    n = rec["n"]
    d = oracle.gen_hostmem(n, np.float32, rec["seed"])
    x3 = np.zeros(16 * n, np.float32)
    inc = ctx.plf(d["x1"], d["x2"], x3, d["EV"], n, d["left"], d["right"], d["wgt"])
    assert hashlib.sha256(x3.tobytes()).hexdigest() == rec["x3_sha256"]
    assert inc == rec["scalerIncrement"]


def test_plf_f32_aie_kat(ctx):
    k = golden("aie_kat.npz")
    n = 64  # the AIE window holds 64 identical sites per lane
    x1, x2 = np.tile(k["x1"], n), np.tile(k["x2"], n)
    x3 = np.zeros(16 * n, np.float32)
    inc = ctx.plf(x1, x2, x3, k["EV"], n, k["left"], k["right"], np.ones(n, np.int32))
    g = k["golden"]
    nz = g != 0
    for s in range(n):
        site = x3[16 * s:16 * s + 16]
        assert np.array_equal(site[nz], g[nz])
        assert np.all(np.abs(site[~nz]) <= 1e-6)
    assert inc == 0


def test_plf_f32_edge_sites(ctx):
    g = golden("edge_f32.npz")
    n = g["x1"].size // 16
    x3 = np.zeros(16 * n, np.float32)
    inc = ctx.plf(g["x1"], g["x2"], x3, g["EV"], n, g["left"], g["right"], g["wgt"])
    assert np.array_equal(bits(x3), bits(g["x3"]))
    assert inc == int(g["scalerIncrement"])
    # per-site bytes via the device entry point
    import torch

    t = {k: torch_dev(g[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    o3 = torch.empty_like(t["x1"])
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], sc, s)
    torch.cuda.synchronize()
    assert np.array_equal(sc.cpu().numpy(), g["scaler"])
    assert int(s.item()) == int(g["scalerIncrement"])
    assert np.array_equal(bits(o3.cpu().numpy()), bits(g["x3"]))


@pytest.mark.parametrize("n", [0, 1, 3, 15, 16, 17, 63, 64, 65, 127, 129, 1000, 4097, 65537,
                               (1 << 18) + 37, (1 << 20) + 5, (1 << 21) + 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_plf_host_ragged_sizes(ctx, oracle, n, dtype):
    """The host-array entry (plf()'s shape) at ragged sizes, including sizes that
    it pipelines in 2, 8 and 16 site chunks (H2D of one chunk while the previous
    one downloads): x3 and the scaler sum bit-exact against the oracle."""
    d = oracle.gen_hostmem(max(n, 1), dtype, 11 + n)
    w = ((np.arange(max(n, 1)) * 13) % 9).astype(np.int32)
    x3 = np.full(16 * max(n, 1), 7.0, dtype)
    inc = ctx.plf(d["x1"], d["x2"], x3, d["EV"], n, d["left"], d["right"], w)
    if n == 0:
        assert inc == 0 and np.all(x3 == 7.0)
        return
    e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w)
    assert inc == einc
    assert np.array_equal(bits(x3), bits(e3))
    if dtype == np.float64:
        rel_ok(x3, e3)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_plf_dev_full_size_1M(ctx, oracle, dtype):
    """BASELINE config #2 size (2^20 sites): bit-exact vs the oracle, N/4 scaled
    sites, scaler bytes and sum."""
    import torch

    n = 1 << 20
    d = oracle.gen_hostmem(n, dtype, oracle.SEED)
    e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"], threads=16)
    t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    o3 = torch.empty_like(t["x1"])
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], sc, s)
    torch.cuda.synchronize()
    got = o3.cpu().numpy()
    assert int(s.item()) == einc == n // 4
    assert np.array_equal(sc.cpu().numpy(), esc)
    assert np.array_equal(bits(got), bits(e3))
    if dtype == np.float64:
        rel_ok(got, e3)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_plf_dev_beyond_2g_elements(ctx, oracle, dtype):
    """Maximum sizes: n = 2^27 + 5 sites puts CLV element indices past 2^31
    (the reference's `int` element index would overflow at n >= 2^27); the
    kernels index in 64 bits.  Windows at the start, across 2^27 and at the
    ragged end are checked bit-exactly against the oracle; the weighted scaler
    sum equals the sum over the per-site scaler bytes (size-independent)."""
    import torch

    n = (1 << 27) + 5
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    g = torch.Generator(device="cuda")
    g.manual_seed(31)
    x1 = torch.rand(16 * n, dtype=tdt, device="cuda", generator=g)
    x1.view(n, 16)[0::4] *= 1e-12
    x2 = torch.rand(16 * n, dtype=tdt, device="cuda", generator=g)
    x3 = torch.empty_like(x1)
    EV = torch.rand(16, dtype=tdt, device="cuda", generator=g)
    L = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    R = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    wgt = torch.randint(0, 3, (n,), dtype=torch.int32, device="cuda", generator=g)
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_dev(x1, x2, x3, EV, L, R, wgt, sc, s)
    torch.cuda.synchronize()
    assert int(s.item()) == int((sc.to(torch.int64) * wgt.to(torch.int64)).sum().item())
    assert int(sc.sum().item()) >= n // 4
    h = lambda t: t.cpu().numpy()  # noqa: E731
    for lo in (0, (1 << 27) - 1000, n - 2000):
        m = min(2000, n - lo)
        sl = slice(16 * lo, 16 * (lo + m))
        e3, esc, _ = oracle.plf(h(x1[sl]), h(x2[sl]), h(EV), h(L), h(R), h(wgt[lo:lo + m]))
        assert np.array_equal(bits(h(x3[sl])), bits(e3)), lo
        assert np.array_equal(h(sc[lo:lo + m]), esc), lo
    del x1, x2, x3
    torch.cuda.empty_cache()


def fill_uniform(t, g, chunk=1 << 30):
    """U[0,1) in place, chunk by chunk (one 64-GB tensor in bounded pieces)."""
    flat = t.view(-1)
    for i in range(0, flat.numel(), chunk):
        flat[i:i + chunk].uniform_(generator=g)


@pytest.mark.parametrize("dtype,n", [(np.float32, 1_000_000_000), (np.float64, 500_000_000)])
def test_plf_dev_reference_sweep_maximum(ctx, oracle, dtype, n):
    """The largest ALIGNMENT_SITES of the reference's sweep (Makefile:16: up to
    1e9 sites, in f32) in ONE device call: 1e9 sites f32 and 5e8 sites f64
    (the largest sweep point whose three f64 CLVs fit: 192 GB), each ~197 GB of
    one GPU's 288 GB.  Element indices pass 2^32 (the reference's 32-bit byte
    counts overflow here).  Windows at the start, at the 2^31- and
    2^32-element crossings, in the middle and at the ragged end are bit-exact
    against the oracle; Σ scaler·wgt equals the sum over the per-site scaler
    bytes (chunked, size-independent)."""
    import torch

    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    g = torch.Generator(device="cuda")
    g.manual_seed(97)
    x1 = torch.empty(16 * n, dtype=tdt, device="cuda")
    x2 = torch.empty_like(x1)
    x3 = torch.empty_like(x1)
    try:
        fill_uniform(x1, g)
        fill_uniform(x2, g)
        x1.view(n, 16)[0::4] *= 1e-12
        EV = torch.rand(16, dtype=tdt, device="cuda", generator=g)
        L = torch.rand(64, dtype=tdt, device="cuda", generator=g)
        R = torch.rand(64, dtype=tdt, device="cuda", generator=g)
        wgt = torch.randint(0, 3, (n,), dtype=torch.int32, device="cuda", generator=g)
        sc = torch.empty(n, dtype=torch.uint8, device="cuda")
        s = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctx.plf_dev(x1, x2, x3, EV, L, R, wgt, sc, s)
        torch.cuda.synchronize()
        c = 1 << 26
        tot = sum(int((sc[i:i + c].to(torch.int64) * wgt[i:i + c]).sum().item()) for i in range(0, n, c))
        assert int(s.item()) == tot
        assert sum(int(sc[i:i + c].sum(dtype=torch.int64).item()) for i in range(0, n, c)) >= n // 4
        h = lambda t: t.cpu().numpy()  # noqa: E731
        for lo in (0, (1 << 27) - 1000, (1 << 28) - 1000, n // 2 + 3, n - 2000):
            m = min(2000, n - lo)
            sl = slice(16 * lo, 16 * (lo + m))
            e3, esc, _ = oracle.plf(h(x1[sl]), h(x2[sl]), h(EV), h(L), h(R), h(wgt[lo:lo + m]))
            assert np.array_equal(bits(h(x3[sl])), bits(e3)), lo
            assert np.array_equal(h(sc[lo:lo + m]), esc), lo
    finally:
        del x1, x2, x3
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def segments_ctx(monkeypatch, mode):
    """A context whose node kernels use the XCD-segmented site mapping always
    (mode "1") or never ("0"); the default picks it by size, from 2^25 sites
    up in f32 and f64 (plf_kernels.hip kSegMinSites32 / 64)."""
    import plfx

    monkeypatch.setenv("PLFX_NODE_SEGMENTS", mode)
    try:
        return plfx.Context(0)
    finally:
        monkeypatch.delenv("PLFX_NODE_SEGMENTS")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_plf_dev_xcd_segments_full_compare(ctx, oracle, monkeypatch, dtype):
    """2^24 + 13 sites through both site mappings of the node kernels -- one
    window for the whole chip, and eight segments, one per XCD (plf_dna.hpp
    wave_sites; by default from 2^25 sites, f32 and f64) -- and the default
    choice: the WHOLE x3 and every scaler byte bit-exact against the oracle,
    segment boundaries and the ragged last segment included, with and without
    the in-kernel sum (two kernel instantiations each)."""
    import torch

    n = (1 << 24) + 13
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    g = torch.Generator(device="cuda")
    g.manual_seed(41)
    x1 = torch.rand(16 * n, dtype=tdt, device="cuda", generator=g)
    x1.view(n, 16)[0::4] *= 1e-12
    x2 = torch.rand(16 * n, dtype=tdt, device="cuda", generator=g)
    EV = torch.rand(16, dtype=tdt, device="cuda", generator=g)
    L = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    R = torch.rand(64, dtype=tdt, device="cuda", generator=g)
    wgt = torch.randint(-2, 4, (n,), dtype=torch.int32, device="cuda", generator=g)
    h = lambda t: t.cpu().numpy()  # noqa: E731
    e3, esc, einc = oracle.plf(h(x1), h(x2), h(EV), h(L), h(R), h(wgt), threads=16)
    on, off = segments_ctx(monkeypatch, "1"), segments_ctx(monkeypatch, "0")
    try:
        for label, c in (("default", ctx), ("segments", on), ("one window", off)):
            for with_sum in (True, False):
                x3 = torch.empty_like(x1)
                sc = torch.empty(n, dtype=torch.uint8, device="cuda")
                s = torch.zeros(1, dtype=torch.int64, device="cuda") if with_sum else None
                c.plf_dev(x1, x2, x3, EV, L, R, wgt, sc, s)
                torch.cuda.synchronize()
                assert np.array_equal(bits(h(x3)), bits(e3)), (label, with_sum)
                assert np.array_equal(h(sc), esc), (label, with_sum)
                if with_sum:
                    assert int(s.item()) == einc
                del x3, sc
    finally:
        on.close()
        off.close()
    del x1, x2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [1, 7, 100, 1000, 1025, 4097, 65539, 300001])
def test_plf_dev_xcd_segments_forced_small(ctx, oracle, monkeypatch, n):
    """The segmented mapping forced on at small and ragged sizes, where the
    eight segments are short or ragged (below 8 blocks of work, n <= 1024 f64,
    the one window runs instead): bit-exact against the oracle, f32 and f64,
    scaler sums exact."""
    import torch

    on = segments_ctx(monkeypatch, "1")
    try:
        for dtype in (np.float32, np.float64):
            d = oracle.gen_hostmem(n, dtype, 9)
            e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
            t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
            x3 = torch.empty_like(t["x1"])
            sc = torch.empty(n, dtype=torch.uint8, device="cuda")
            s = torch.zeros(1, dtype=torch.int64, device="cuda")
            on.plf_dev(t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"], t["wgt"], sc, s)
            torch.cuda.synchronize()
            assert np.array_equal(bits(x3.cpu().numpy()), bits(e3))
            assert np.array_equal(sc.cpu().numpy(), esc)
            assert int(s.item()) == einc
    finally:
        on.close()


def _captured_grids(call):
    """[(kernel name, workgroups, workgroup size)] of the launches `call`
    makes, read from the kernel nodes of a captured graph (what the graph
    will dispatch), then the graph is replayed once."""
    import torch

    import bench

    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=st):
        call(st.cuda_stream)
    out = [(name, grid // wg, wg) for name, grid, wg in bench.graph_kernel_launches(g)]
    g.instantiate()
    with torch.cuda.stream(st):
        g.replay()
    torch.cuda.synchronize()
    del g
    return out


@pytest.mark.parametrize("cap", [4, 12])
def test_segment_grid_never_exceeds_block_cap(oracle, monkeypatch, cap):
    """with the segments forced on (PLFX_NODE_SEGMENTS=1)
    and a grid cap (PLFX_MAX_BLOCKS), the node kernel never launches more
    blocks than the cap -- below 8 the one-window mapping runs, at 12 the
    segmented grid is 8 -- and stays bit-exact, f32 and f64, at 2^20 sites
    (where the uncapped grid is far larger).  Invalid env values are refused."""
    import torch

    import plfx

    monkeypatch.setenv("PLFX_MAX_BLOCKS", str(cap))
    monkeypatch.setenv("PLFX_NODE_SEGMENTS", "1")
    c = plfx.Context(0)
    monkeypatch.delenv("PLFX_MAX_BLOCKS")
    monkeypatch.delenv("PLFX_NODE_SEGMENTS")
    n = 1 << 20
    try:
        for dtype in (np.float32, np.float64):
            d = oracle.gen_hostmem(n, dtype, 17)
            e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
            t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
            x3 = torch.empty_like(t["x1"])
            sc = torch.empty(n, dtype=torch.uint8, device="cuda")
            s = torch.zeros(1, dtype=torch.int64, device="cuda")
            grids = _captured_grids(lambda sh: c.plf_dev(t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"],
                                                         t["wgt"], sc, s, stream=sh))
            node = [x for x in grids if x[0] and "plf_dna" in x[0]]
            assert len(node) == 1, grids
            assert node[0][1] == (8 if cap >= 8 else cap), grids
            assert np.array_equal(bits(x3.cpu().numpy()), bits(e3))
            assert np.array_equal(sc.cpu().numpy(), esc) and int(s.item()) == einc
            del t, x3, sc, s
    finally:
        c.close()
    for bad in ("2", "yes", "on"):
        monkeypatch.setenv("PLFX_NODE_SEGMENTS", bad)
        with pytest.raises(Exception):
            plfx.Context(0)
    for good in ("auto", "-1", "0"):
        monkeypatch.setenv("PLFX_NODE_SEGMENTS", good)
        plfx.Context(0).close()
    monkeypatch.delenv("PLFX_NODE_SEGMENTS")


@pytest.mark.parametrize("streams", [2, 3])
def test_streams_setting_grids_and_bits(oracle, monkeypatch, streams):
    """plfx_ctx_set_streams (bench.py lanes): with `streams` one-node calls in
    flight the dense DNA node kernels (f32, f64) and the f64 protein FMA
    kernel launch the resident blocks / streams -- the captured grids say so
    -- and give the same bits as with 1, also with `streams` calls running at
    once on as many streams; other values and bad PLFX_STREAMS are refused."""
    import torch

    import plfx

    c = plfx.Context(0)
    try:
        assert c.streams == 1
        for bad in (0, plfx.STREAMS_MAX + 1, -1):
            with pytest.raises(plfx.PlfxError):
                c.set_streams(bad)
        assert c.streams == 1
        n = 1 << 20
        for dtype in (np.float32, np.float64):
            d = oracle.gen_hostmem(n, dtype, 23 + streams)
            e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"],
                                       threads=16)
            t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
            outs = [(torch.empty_like(t["x1"]), torch.empty(n, dtype=torch.uint8, device="cuda"),
                     torch.zeros(1, dtype=torch.int64, device="cuda")) for _ in range(streams)]

            def call(sh, o=outs[0]):
                c.plf_dev(t["x1"], t["x2"], o[0], t["EV"], t["left"], t["right"], t["wgt"], o[1], o[2],
                          stream=sh)

            grids = {}
            for k in (1, streams):
                c.set_streams(k)
                grids[k] = [g for g in _captured_grids(call) if g[0] and "plf_dna" in g[0]]
                assert len(grids[k]) == 1, grids
            assert grids[streams][0][1] == grids[1][0][1] // streams, grids
            # `streams` calls at once, one per stream, on the smaller grids
            sts = [torch.cuda.Stream() for _ in range(streams)]
            torch.cuda.synchronize()
            for o, st_ in zip(outs, sts):
                call(st_.cuda_stream, o)
            torch.cuda.synchronize()
            for o in outs:
                assert np.array_equal(bits(o[0].cpu().numpy()), bits(e3))
                assert np.array_equal(o[1].cpu().numpy(), esc) and int(o[2].item()) == einc
            for st_ in sts:
                c.release_stream(st_)
            c.set_streams(1)
            del t, outs
        # a DNA batch (plfx_plf_batch_dev) shares the grid the same way (its
        # own context: every captured stream keeps a pool workspace)
        cb = plfx.Context(0)
        try:
            nb = 1 << 18
            d = oracle.gen_hostmem(nb, np.float64, 31)
            e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
            t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
            bnodes = [dict(x1=t["x1"], x2=t["x2"], x3=torch.empty_like(t["x1"]), left=t["left"],
                           right=t["right"], scaler=torch.empty(nb, dtype=torch.uint8, device="cuda"),
                           scaler_sum=torch.zeros(1, dtype=torch.int64, device="cuda")) for _ in range(2)]
            bgrid = {}
            for k in (1, streams):
                cb.set_streams(k)
                g = [x for x in _captured_grids(lambda sh: cb.plf_batch_dev(bnodes, t["EV"], nb, t["wgt"],
                                                                            stream=sh))
                     if x[0] and "batch" in x[0]]
                assert len(g) == 1, g
                bgrid[k] = g[0][1]  # workgroups over both nodes
                for nd in bnodes:
                    assert np.array_equal(bits(nd["x3"].cpu().numpy()), bits(e3))
                    assert np.array_equal(nd["scaler"].cpu().numpy(), esc)
                    assert int(nd["scaler_sum"].item()) == einc
            assert bgrid[streams] == (bgrid[1] // 2 // streams) * 2, bgrid
            del t, bnodes
        finally:
            cb.close()
        # protein f64 FMA (matrix cores): same bits at 1 and `streams`
        m = 1 << 18
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        x1 = torch.rand(m * 80, dtype=torch.float64, device="cuda", generator=g)
        x1.view(-1, 80)[0::4] *= 1e-14
        x2 = torch.rand(m * 80, dtype=torch.float64, device="cuda", generator=g)
        EV = torch.rand(400, dtype=torch.float64, device="cuda", generator=g) - 0.25
        P = torch.rand(3200, dtype=torch.float64, device="cuda", generator=g)
        res = {}
        for k in (1, streams):
            c.set_streams(k)
            x3 = torch.empty_like(x1)
            sc = torch.empty(m, dtype=torch.uint8, device="cuda")
            ss = torch.zeros(1, dtype=torch.int64, device="cuda")

            def pcall(sh):
                c.plf_dev_gen(x1, x2, x3, EV, P[:1600], P[1600:], 20, None, sc, ss, fma=True, stream=sh)

            pg = [x for x in _captured_grids(pcall) if x[0] and "plf_prot_mfma" in x[0]]
            assert len(pg) == 1, pg
            res[k] = (pg[0][1], x3.cpu().numpy(), sc.cpu().numpy(), int(ss.item()))
        assert res[streams][0] == res[1][0] // streams
        assert np.array_equal(bits(res[1][1]), bits(res[streams][1]))
        assert np.array_equal(res[1][2], res[streams][2]) and res[1][3] == res[streams][3] > 0
        # protein f32 FMA: whole blocks per CU, rounded up (3 per CU -> 2 at 2 streams)
        x1f, x2f = x1.float(), x2.float()
        EVf, Pf = EV.float(), P.float()
        resf = {}
        for k in (1, streams):
            c.set_streams(k)
            x3 = torch.empty_like(x1f)
            sc = torch.empty(m, dtype=torch.uint8, device="cuda")
            ss = torch.zeros(1, dtype=torch.int64, device="cuda")

            def fcall(sh):
                c.plf_dev_gen(x1f, x2f, x3, EVf, Pf[:1600], Pf[1600:], 20, None, sc, ss, fma=True, stream=sh)

            fg = [x for x in _captured_grids(fcall) if x[0] and "plf_prot_mfma32" in x[0]]
            assert len(fg) == 1, fg
            resf[k] = (fg[0][1], x3.cpu().numpy(), sc.cpu().numpy(), int(ss.item()))
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        per_cu = resf[1][0] // ncu
        assert resf[streams][0] == ncu * -(-per_cu // streams)
        assert np.array_equal(bits(resf[1][1]), bits(resf[streams][1]))
        assert np.array_equal(resf[1][2], resf[streams][2]) and resf[1][3] == resf[streams][3] > 0
    finally:
        c.close()
    monkeypatch.setenv("PLFX_STREAMS", str(streams))
    monkeypatch.setenv("PLFX_NODE_SEGMENTS", "1")  # the XCD-segmented mapping on the smaller grid
    c = plfx.Context(0)
    monkeypatch.delenv("PLFX_NODE_SEGMENTS")
    try:
        assert c.streams == streams
        n = 1 << 20
        d = oracle.gen_hostmem(n, np.float64, 5)
        e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"], threads=16)
        t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
        x3 = torch.empty_like(t["x1"])
        sc = torch.empty(n, dtype=torch.uint8, device="cuda")
        s = torch.zeros(1, dtype=torch.int64, device="cuda")
        g = [x for x in _captured_grids(lambda sh: c.plf_dev(t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"],
                                                             t["wgt"], sc, s, stream=sh)) if x[0] and "plf_dna" in x[0]]
        assert len(g) == 1 and g[0][1] % 8 == 0 and g[0][1] <= 1024 // streams, g
        assert np.array_equal(bits(x3.cpu().numpy()), bits(e3))
        assert np.array_equal(sc.cpu().numpy(), esc) and int(s.item()) == einc
    finally:
        c.close()
    for bad in ("0", "9", "x", "12", " 2"):
        monkeypatch.setenv("PLFX_STREAMS", bad)
        with pytest.raises(Exception):
            plfx.Context(0)
    monkeypatch.setenv("PLFX_STREAMS", "")
    c = plfx.Context(0)
    assert c.streams == 1
    c.close()
    monkeypatch.delenv("PLFX_STREAMS")


def test_plf_dev_repeated_calls_and_optional_outputs(ctx, oracle):
    """The in-kernel ticket reduction resets itself: back-to-back launches with
    different weights each report their own sum; outputs are optional."""
    import torch

    n = 300_001
    d = oracle.gen_hostmem(n, np.float64, 5)
    t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right")}
    o3 = torch.empty_like(t["x1"])
    sums = torch.zeros(6, dtype=torch.int64, device="cuda")
    ws = [np.full(n, i + 1, np.int32) for i in range(5)]
    wt = [torch_dev(w) for w in ws]
    for i in range(5):
        ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], wt[i], None, sums[i:i + 1])
    ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], None, None, sums[5:6])
    ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"])  # no scaler outputs
    torch.cuda.synchronize()
    n_sc = -(-n // 4)
    assert sums.cpu().tolist() == [n_sc * (i + 1) for i in range(5)] + [n_sc]
    e3, _, _ = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"])
    assert np.array_equal(bits(o3.cpu().numpy()), bits(e3))


def test_plf_dev_nonfinite_and_signed(ctx, oracle):
    """NaN/inf inputs propagate like the CPU path and never scale; negative
    CLV entries (cancellation in the EV transform)."""
    import torch

    n = 4096
    rng = np.random.default_rng(1)
    d = oracle.gen_hostmem(n, np.float64, 3)
    x1 = d["x1"].copy()
    x1[rng.integers(0, x1.size, 50)] = np.nan
    x1[rng.integers(0, x1.size, 50)] = np.inf
    EV = (rng.random(16) - 0.5)
    left = rng.random(64) - 0.3
    e3, esc, einc = oracle.plf(x1, d["x2"], EV, left, d["right"])
    t = [torch_dev(a) for a in (x1, d["x2"], EV, left, d["right"])]
    o3 = torch.empty_like(t[0])
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_dev(t[0], t[1], o3, t[2], t[3], t[4], None, sc, s)
    torch.cuda.synchronize()
    got = o3.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(e3))
    m = ~np.isnan(e3)
    assert np.array_equal(bits(got[m]), bits(e3[m]))
    assert np.array_equal(sc.cpu().numpy(), esc) and int(s.item()) == einc


def test_scaler_sum_kernel(ctx, oracle):
    import torch

    for n in (0, 1, 255, 256, 257, 1_000_003):
        sc = (np.arange(n) % 3 == 1).astype(np.uint8)
        w = ((np.arange(n) * 7) % 11 - 3).astype(np.int32)  # negative weights too
        out = torch.full((2,), -1, dtype=torch.int64, device="cuda")
        ctx.scaler_sum(torch_dev(sc), torch_dev(w), out[0:1], n=n)
        ctx.scaler_sum(torch_dev(sc), None, out[1:2], n=n)
        torch.cuda.synchronize()
        assert out.cpu().tolist() == [oracle.scaler_sum(sc, w), oracle.scaler_sum(sc)]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("layout,P,W,aie", [(0, 1, 8192, 1), (1, 1, 8192, 1), (0, 3, 1024, 1),
                                            (1, 4, 16288, 1), (1, 2, 0, 0)])
def test_instance_run_contract(ctx, oracle, dtype, layout, P, W, aie):
    """The accelerator buffer contract: reference packing per instance, kernel
    reads the header in place, writes exactly n_k CLVs and scaler bytes and
    never the window padding."""
    import plfx
    import torch

    n = 5000
    d = oracle.gen_hostmem(n, dtype, 21)
    tb = plfx.Testbench(n, P, W if W else 1024, layout, aie)
    e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    out = np.empty(16 * n, dtype)
    scal = np.empty(n, np.uint8)
    for k in range(P):
        nk = tb.alignments_per_instance(k)
        off = tb.instance_site_offset(k)
        L, R = tb.pack_instance(k, d["EV"], d["left"], d["right"], d["x1"], d["x2"])
        dL, dR = torch_dev(L), torch_dev(R)
        dO = torch.full((tb.instance_elements_out(),), -3.0, dtype=dL.dtype, device="cuda")
        dS = torch.full((nk + 64,), 0xAB, dtype=torch.uint8, device="cuda")
        ctx.instance_run(dL, dR, dO, dS, nk, W, layout)
        torch.cuda.synchronize()
        o = dO.cpu().numpy()
        sb = dS.cpu().numpy()
        assert np.all(o[16 * nk:] == -3.0)       # padding untouched
        assert np.all(sb[nk:] == 0xAB)
        out[16 * off:16 * (off + nk)] = o[:16 * nk]
        scal[off:off + nk] = sb[:nk]
    assert np.array_equal(bits(out), bits(e3))
    assert np.array_equal(scal, esc)
    # host reduction (host_mem.cpp:384-388)
    assert int((scal.astype(np.int64) * d["wgt"]).sum()) == einc


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("layout,P,W", [(0, 3, 1024), (1, 4, 16288), (1, 1, 8192)])
def test_instance_run_host_buffers(ctx, oracle, dtype, layout, P, W):
    """The instance contract on host buffers (bo.write -> run -> bo.read):
    the reference's packed bos in, n_k CLVs and scaler bytes out, bit-exact,
    nothing written past n_k."""
    import plfx

    n = 4099
    d = oracle.gen_hostmem(n, dtype, 23)
    tb = plfx.Testbench(n, P, W, layout, 1)
    e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    out = np.empty(16 * n, dtype)
    scal = np.empty(n, np.uint8)
    for k in range(P):
        nk = tb.alignments_per_instance(k)
        off = tb.instance_site_offset(k)
        L, R = tb.pack_instance(k, d["EV"], d["left"], d["right"], d["x1"], d["x2"])
        o = np.full(tb.instance_elements_out(), -3.0, dtype)
        sb = np.full(nk + 64, 0xAB, np.uint8)
        ctx.instance_run_host(L, R, o, sb, nk, W, layout)
        assert np.all(o[16 * nk:] == -3.0) and np.all(sb[nk:] == 0xAB)
        out[16 * off:16 * (off + nk)] = o[:16 * nk]
        scal[off:off + nk] = sb[:nk]
    assert np.array_equal(bits(out), bits(e3))
    assert np.array_equal(scal, esc)
    assert int((scal.astype(np.int64) * d["wgt"]).sum()) == einc


@pytest.mark.parametrize("n", [1, 4099, (1 << 16) + 3])
def test_plf_f64_against_reference_double_instantiation(ctx, oracle, n):
    """The f64 kernels against the REFERENCE's own loop in double (plf.cpp
    compiled with float spelled double, oracle/_ref/libplfref_f64_O0.so,
    which travels with the snapshot): the device entry (lane-pair kernel) and
    the host plf()-shaped entry, bit for bit, scaler sum exact; every 4th site
    underflows."""
    import torch

    if oracle.ref_lib_f64("O0") is None:
        pytest.skip("oracle/_ref has no f64 build")
    d = oracle.gen_hostmem(n, np.float64, 2024 + n)
    d["x1"].reshape(-1, 16)[::4] *= 1e-30
    w = (np.arange(n) % 7 + 1).astype(np.int32)
    r3, rinc = oracle.ref_plf_f64(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w)
    t = {k: torch_dev(d[k]) for k in ("x1", "x2", "EV", "left", "right")}
    x3 = torch.empty_like(t["x1"])
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.plf_dev(t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"], torch_dev(w), None, s)
    torch.cuda.synchronize()
    assert np.array_equal(bits(x3.cpu().numpy()), bits(r3))
    assert int(s.item()) == rinc
    h3 = np.empty_like(d["x1"])
    inc = ctx.plf(d["x1"], d["x2"], h3, d["EV"], n, d["left"], d["right"], w)
    assert np.array_equal(bits(h3), bits(r3)) and inc == rinc


def test_rejects_bad_arguments(ctx):
    import plfx
    import torch

    x = torch.zeros(16 * 8 + 4, dtype=torch.float32, device="cuda")
    with pytest.raises(plfx.PlfxError) as ei:
        ctx.plf_dev(x[1:129], x[:128], x[:128].clone(), x[:16], x[:64], x[:64])  # misaligned
    assert ei.value.code == plfx.ERR_INVALID
    y = torch.zeros(128, dtype=torch.float32, device="cuda")
    with pytest.raises(plfx.PlfxError):
        ctx.plf_dev(y, y.clone(), y, y[:16], y[:64], y[:64])  # x3 aliases x1


def test_host_driver_end_to_end(oracle, tmp_path):
    """plfx_host (the host_mem.cpp counterpart): H2D left || H2D right ->
    kernel -> D2H CLV || D2H scaler per instance on two streams joined by
    events; dumped CLVs/scalers equal the oracle on the same host_mem-protocol
    inputs (std::mt19937, same seed).  --no-intermediate is the reference's
    NO_INTERMEDIATE_RESULTS mode (host_mem.cpp:327-392,454-468) and --csv its
    write_to_csv (timing.h:153-194); --devices spreads the instances over a
    GPU list, one context per entry; --reduce rccl replaces the host scaler
    loop by per-instance device sums and ONE RCCL all-reduce."""
    exe = PKG / "build" / "plfx_host"
    assert exe.exists()
    cases = ((np.float32, ["--dtype", "f32", "--layout", "comb", "--window", "1024"], False),
             (np.float64, ["--dtype", "f64", "--layout", "sep", "--window", "8192"], False),
             (np.float64, ["--dtype", "f64", "--layout", "comb", "--window", "8192"], True),
             (np.float32, ["--dtype", "f32", "--layout", "sep", "--window", "1024"], True),
             # instances over a GPU list (one context per entry; the box has one GPU,
             # so two contexts on it): instances 0 and 2 on context 0, 1 on context 1
             (np.float64, ["--dtype", "f64", "--layout", "sep", "--window", "8192", "--devices", "0,0"], False),
             (np.float32, ["--dtype", "f32", "--layout", "comb", "--window", "1024", "--devices", "0,0"], True),
             # the scaler totals through ONE RCCL all-reduce (world 1 on the box)
             # instead of the host loop, in both run modes
             (np.float64, ["--dtype", "f64", "--layout", "sep", "--window", "8192", "--devices", "0",
                           "--reduce", "rccl"], False),
             (np.float64, ["--dtype", "f64", "--layout", "comb", "--window", "8192", "--reduce", "rccl"], True))
    for ci, (dtype, args, noint) in enumerate(cases):
        n, calls, P = 3001, 2, 3
        pre = str(tmp_path / f"out{ci}_{np.dtype(dtype).name}")
        csv = tmp_path / f"t{ci}.csv"
        extra = ["--no-intermediate"] if noint else []
        r = subprocess.run([str(exe), str(n), str(calls), str(P), *args, *extra, "--dump", pre,
                            "--csv", str(csv)], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        d = oracle.gen_hostmem(n, dtype, oracle.SEED)
        e3, esc, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
        for i in range(calls):
            got = np.fromfile(f"{pre}_call{i}_x3.bin", dtype=dtype)
            sc = np.fromfile(f"{pre}_call{i}_scaler.bin", dtype=np.uint8)
            inc = int(open(f"{pre}_call{i}_inc.txt").read())
            assert np.array_equal(bits(got), bits(e3))
            assert np.array_equal(sc, esc) and inc == einc
        lines = csv.read_text().strip().split("\n")
        assert len(lines) == 1 + calls
        if noint:
            for row in ("Prepare input for GPU:", "PLF on GPU:", "scaling wgt mult:"):
                assert row in r.stdout
            assert "GPU PLF kernel" not in r.stdout
            assert lines[0] == "preparation,plf,scaling"
        else:
            assert "GPU PLF kernel" in r.stdout and "[all instances] Host to GPU memory" in r.stdout
            assert lines[0].split(",") == ([f"hm{k}" for k in range(P)] + [f"msasm{k}" for k in range(P)]
                                           + [f"mh{k}" for k in range(P)])
        for ln in lines[1:]:
            vals = [float(v) for v in ln.split(",")]
            assert len(vals) == len(lines[0].split(",")) and all(v >= 0 for v in vals)
        # the report's sizing rows (host_mem.cpp:56-88): instances, buffers, all calls, memory
        check_report_rows(r.stdout, n, calls, P, dtype, args)
        assert "RAM usage (GPU):" in r.stdout and " GB of " in r.stdout.split("RAM usage (GPU):")[1]
        # the driver's own check (host_mem.cpp:403-442): CPU plf() vs the GPU, exact
        assert "Test result: Passed" in r.stdout
        assert "Reference (CPU plf" in r.stdout and "Speed up (excluding transfers)" in r.stdout
        assert ("reduce = rccl (1 rank, RCCL " if "rccl" in args else "reduce = host (") in r.stdout
    bad = subprocess.run([str(exe), "3001", "1", "2", "--devices", "0,0", "--reduce", "rccl"],
                         capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "distinct GPUs" in bad.stderr  # refused, not a silent host sum


def test_dropin_header_reference_call(tmp_path):
    """A C++ call site written exactly like host_mem.cpp:418, compiled against
    include/plfx_plf.hpp, reproduces the reference fixture bit for bit."""
    from test_abi import build_dropin

    g = golden("hostmem_f32_n1000.npz")
    n = 1000
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(np.int32(n).tobytes())
        for k in ("EV", "left", "right", "x1", "x2"):
            f.write(np.ascontiguousarray(g[k], np.float32).tobytes())
        f.write(np.ascontiguousarray(g["wgt"], np.int32).tobytes())
    exe = build_dropin(tmp_path)
    out = tmp_path / "out.bin"
    r = subprocess.run([str(exe), str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.uint8)
    x3 = raw[:64 * n].view(np.float32)
    inc = int(raw[64 * n:].view(np.int32)[0])
    assert np.array_equal(bits(x3), bits(g["x3"]))
    assert inc == int(g["scalerIncrement"])
