"""GPU tests of the C ABI's concurrency and capture rules (plfx.h "Streams and
the scaler-sum workspace") and of the configurations the bench times at their
benchmarked sizes: protein FMA at 2^18 sites (BASELINE configs[4]) and 64
batched nodes x 2^20 sites (configs[3]'s per-GPU shard).  Bar: CLVs, scaler
bytes and sums bit-exact against the oracle; protein FMA also within 1e-12
(relative to the site's largest value) of the unfused loop."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_sums_on_two_streams_concurrently(ctx, oracle):
    """Sum-producing launches in flight on two streams of ONE context at the
    same time (each stream has its own reduction workspace): every sum exact,
    the CLVs bit-exact.  Also the root lnL on both streams."""
    import torch

    n = 1 << 20
    d = oracle.gen_hostmem(n, np.float64, 41)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right")}
    ws = [dev(np.full(n, i + 1, np.int32)) for i in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.empty_like(t["x1"]) for _ in range(2)]
    sums = torch.zeros(2, 8, dtype=torch.int64, device="cuda")
    lnl = torch.zeros(2, 8, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for r in range(8):  # interleaved issue: both streams' kernels overlap on the device
        for i, s in enumerate(streams):
            ctx.plf_dev(t["x1"], t["x2"], outs[i], t["EV"], t["left"], t["right"], ws[i], None,
                        sums[i, r:r + 1], stream=s)
            ctx.root_lnl(outs[i], n, lnl[i, r:r + 1], wgt=ws[i], scaler_sums=sums[i, r:r + 1],
                         stream=s)
    torch.cuda.synchronize()
    n_sc = n // 4
    assert sums[0].tolist() == [n_sc] * 8 and sums[1].tolist() == [2 * n_sc] * 8
    e3, _, _ = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], threads=16)
    for o in outs:
        assert np.array_equal(bits(o.cpu().numpy()), bits(e3))
    l0 = oracle.root_lnl(4, 4, e3, n, wgt=np.ones(n, np.int32), scaler_sums=np.array([n_sc]))
    got = lnl.cpu().numpy()
    assert np.all(np.abs(got[0] - l0) <= 1e-12 * abs(l0))
    assert np.all(got[0] == got[0][0]) and np.all(got[1] == got[1][0])  # deterministic


def test_one_context_from_several_host_threads(ctx, oracle):
    """plfx.h: calls on one context from several host threads are serialised by
    the context.  Four Python threads (ctypes drops the GIL for each call), each
    on its own stream, issue node updates with scaler sums and root lnLs on the
    SAME context at once: every sum exact, every CLV bit-exact, lnL identical."""
    import threading

    import torch

    n = 1 << 18
    d = oracle.gen_hostmem(n, np.float64, 43)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right")}
    nt, reps = 4, 16
    ws = [dev(np.full(n, i + 1, np.int32)) for i in range(nt)]
    outs = [torch.empty_like(t["x1"]) for _ in range(nt)]
    sums = torch.zeros(nt, reps, dtype=torch.int64, device="cuda")
    lnl = torch.zeros(nt, reps, dtype=torch.float64, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(nt)]
    torch.cuda.synchronize()
    errs = []
    go = threading.Barrier(nt)

    def worker(i):
        try:
            go.wait()
            for r in range(reps):
                ctx.plf_dev(t["x1"], t["x2"], outs[i], t["EV"], t["left"], t["right"], ws[i], None,
                            sums[i, r:r + 1], stream=streams[i])
                ctx.root_lnl(outs[i], n, lnl[i, r:r + 1], wgt=ws[i], scaler_sums=sums[i, r:r + 1],
                             stream=streams[i])
            streams[i].synchronize()
        except Exception as e:  # reported on the main thread
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(nt)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=60)
    assert not errs, errs
    torch.cuda.synchronize()
    n_sc = n // 4
    for i in range(nt):
        assert sums[i].tolist() == [(i + 1) * n_sc] * reps
    e3, _, _ = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], threads=16)
    for o in outs:
        assert np.array_equal(bits(o.cpu().numpy()), bits(e3))
    got = lnl.cpu().numpy()
    for i in range(nt):
        assert np.all(got[i] == got[i][0])
    assert np.allclose(got[1], 2 * got[0], rtol=1e-12)  # weights 2 vs 1: lnL doubles


def test_host_entry_from_several_threads(ctx, oracle):
    """The synchronous plf() entry stages through ONE device buffer per context:
    four threads calling it on the same context at once (different inputs) must
    each get exactly their own reference result (the per-context lock)."""
    import threading

    n = 200_003
    ins = [oracle.gen_hostmem(n, np.float64, 60 + i) for i in range(4)]
    want = [oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], threads=4) for d in ins]
    outs = [np.empty_like(d["x1"]) for d in ins]
    incs = [None] * 4
    errs = []
    go = threading.Barrier(4)

    def worker(i):
        try:
            d = ins[i]
            go.wait()
            for _ in range(3):
                incs[i] = ctx.plf(d["x1"], d["x2"], outs[i], d["EV"], n, d["left"], d["right"], None)
        except Exception as e:  # reported on the main thread
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    for i in range(4):
        e3, _, inc = want[i]
        assert np.array_equal(bits(outs[i]), bits(e3))
        assert incs[i] == inc


def _hip():
    import ctypes

    import torch  # noqa: F401 -- the HIP runtime torch already loaded

    return ctypes.CDLL("libamdhip64.so")


def _new_streams(k):
    import ctypes

    hip = _hip()
    out = []
    for _ in range(k):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # hipStreamNonBlocking
        out.append(h.value)
    return out


def _destroy_streams(hs):
    import ctypes

    hip = _hip()
    for h in hs:
        assert hip.hipStreamDestroy(ctypes.c_void_p(h)) == 0


# the rejected capture below ends with an empty graph, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
def test_graph_capture_first_use_from_the_pool(oracle):
    """The first PLFX_WS_POOL streams take workspaces allocated with the
    context, so a stream's FIRST sum-producing call may be inside a capture;
    once the pool is used up, a cold stream's first call inside a capture is
    rejected with PlfxError (its workspace would be allocated then), and a
    stream warmed outside captures fine.  Replays give exact sums."""
    import plfx
    import torch

    n = 70001
    d = oracle.gen_hostmem(n, np.float64, 43)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    e3, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    with plfx.Context(0) as c:
        o3 = torch.empty_like(t["x1"])
        s = torch.zeros(1, dtype=torch.int64, device="cuda")
        cold = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cold):  # cold stream, pool entry: fine
            for _ in range(3):
                c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s,
                          stream=cold)
        s.zero_()
        torch.cuda.synchronize()
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
        assert int(s.item()) == einc
        assert np.array_equal(bits(o3.cpu().numpy()), bits(e3))
        # use up the pool (`cold` holds one entry)
        hs = _new_streams(plfx.WS_POOL - 1)
        sums = torch.zeros(len(hs), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        for i, h in enumerate(hs):
            c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None,
                      sums[i:i + 1], stream=h)
        torch.cuda.synchronize()
        late = torch.cuda.Stream()
        g2 = torch.cuda.CUDAGraph()
        with pytest.raises(plfx.PlfxError):
            with torch.cuda.graph(g2, stream=late):
                c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s,
                          stream=late)
        for h in hs:
            c.release_stream(h)
        _destroy_streams(hs)
        assert sums.tolist() == [einc] * len(hs)


def test_per_thread_default_stream_from_threads(oracle):
    """hipStreamPerThread is ONE handle value naming a different stream in every
    host thread: each thread gets its own workspace, so four
    threads issuing sum-producing calls on it at once all get exact sums."""
    import threading

    import plfx
    import torch

    n = 1 << 18
    d = oracle.gen_hostmem(n, np.float64, 47)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right")}
    nt, reps = 4, 24
    ws = [dev(np.full(n, i + 1, np.int32)) for i in range(nt)]
    outs = [torch.empty_like(t["x1"]) for _ in range(nt)]
    sums = torch.zeros(nt, reps, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    errs = []
    go = threading.Barrier(nt)
    with plfx.Context(0) as c:
        def worker(i):
            try:
                go.wait()
                for r in range(reps):
                    c.plf_dev(t["x1"], t["x2"], outs[i], t["EV"], t["left"], t["right"], ws[i], None,
                              sums[i, r:r + 1], stream=plfx.STREAM_PER_THREAD)
                c.release_stream(plfx.STREAM_PER_THREAD)  # waits for this thread's stream
            except Exception as e:  # reported on the main thread
                errs.append(e)

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nt)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=60)
    assert not errs, errs
    torch.cuda.synchronize()
    n_sc = n // 4
    for i in range(nt):
        assert sums[i].tolist() == [(i + 1) * n_sc] * reps
    e3, _, _ = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], threads=16)
    for o in outs:
        assert np.array_equal(bits(o.cpu().numpy()), bits(e3))


def test_release_stream_recycles_workspaces(oracle):
    """Streams hold a workspace until plfx_ctx_release_stream: more than
    PLFX_MAX_STREAMS streams used one after another work when each is released;
    without releases the (MAX_STREAMS+1)-th is refused until one is released.
    Destroying the context with streams still holding workspaces waits for
    those streams, so the sums are complete after close()."""
    import plfx
    import torch

    n = 4099
    d = oracle.gen_hostmem(n, np.float64, 48)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    _, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    k = plfx.MAX_STREAMS + 6
    hs = _new_streams(k)
    sums = torch.zeros(k, dtype=torch.int64, device="cuda")
    o3 = torch.empty_like(t["x1"])
    torch.cuda.synchronize()

    def call(c, i):
        c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None,
                  sums[i:i + 1], stream=hs[i])

    with plfx.Context(0) as c:  # rotate with releases: never more than one held
        for i in range(k):
            call(c, i)
            c.release_stream(hs[i])
        assert sums.tolist() == [einc] * k
    sums.zero_()
    torch.cuda.synchronize()
    c = plfx.Context(0)
    held = plfx.MAX_STREAMS
    for i in range(held):
        call(c, i)
    with pytest.raises(plfx.PlfxError) as ei:
        call(c, held)
    assert ei.value.code == plfx.ERR_INVALID
    c.release_stream(hs[0])
    call(c, held)
    c.close()  # streams still hold workspaces: destroy waits for the device
    assert sums[1:held + 1].tolist() == [einc] * held
    _destroy_streams(hs)


def test_context_keeps_callers_device(ctx):
    """Entry points bind the context's device and give the caller's current
    device back (one visible GPU: the current device stays 0 across calls)."""
    import plfx
    import torch

    before = torch.cuda.current_device()
    with plfx.Context(0) as c:
        x = torch.zeros(16 * 64, dtype=torch.float64, device="cuda")
        c.plf_dev(x, x.clone(), torch.empty_like(x), x[:16], x[:64], x[:64])
        torch.cuda.synchronize()
    assert torch.cuda.current_device() == before


def test_protein_fma_full_size_256k(ctx, oracle):
    """BASELINE configs[4] in the mode the bench times (FMA, f64 matrix cores)
    at its size, 2^18 sites: bit-exact against the oracle's fma() restatement,
    within 1e-12 of the unfused loop, identical scaler decisions."""
    import torch

    S, CAT, n = 20, 4, 1 << 18
    V = S * CAT
    rng = np.random.default_rng(2026)
    x1 = rng.random(V * n)
    x1.reshape(n, V)[0::4] *= 1e-14
    x2 = rng.random(V * n)
    left, right = rng.random(CAT * S * S), rng.random(CAT * S * S)
    EV = rng.random(S * S) - 0.25
    w = rng.integers(0, 4, n).astype(np.int32)
    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    x3 = torch.empty(V * n, dtype=torch.float64, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, t[5], sc, s, n=n, fma=True)
    torch.cuda.synchronize()
    got, gsc = x3.cpu().numpy(), sc.cpu().numpy()
    f3, fsc, finc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    assert np.array_equal(bits(got), bits(f3))
    assert np.array_equal(gsc, fsc) and int(s.item()) == finc
    e3, esc, einc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w)
    assert np.array_equal(gsc, esc) and finc == einc
    scale = np.abs(e3).reshape(n, V).max(axis=1, keepdims=True)
    assert (np.abs(got - e3).reshape(n, V) / scale).max() <= 1e-12


def test_protein_f32_fma_full_size_256k(ctx, oracle):
    """The f32 protein FMA kernel (matrix cores, rows 16..19 on the 4x4x1 form
    with permlane transposes) at configs[4]'s size, 2^18 sites: bit-exact
    against the oracle's fmaf restatement, scaler bytes and sum included."""
    import torch

    S, CAT, n = 20, 4, 1 << 18
    V = S * CAT
    rng = np.random.default_rng(2027)
    x1 = rng.random(V * n).astype(np.float32)
    x1.reshape(n, V)[1::4] *= np.float32(1e-14)
    x2 = rng.random(V * n).astype(np.float32)
    left = rng.random(CAT * S * S).astype(np.float32)
    right = rng.random(CAT * S * S).astype(np.float32)
    EV = (rng.random(S * S) - 0.25).astype(np.float32)
    w = rng.integers(0, 4, n).astype(np.int32)
    t = [dev(a) for a in (x1, x2, EV, left, right, w)]
    x3 = torch.empty(V * n, dtype=torch.float32, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    ctx.plf_dev_gen(t[0], t[1], x3, t[2], t[3], t[4], S, t[5], sc, s, n=n, fma=True)
    torch.cuda.synchronize()
    f3, fsc, finc = oracle.plf_generic(S, CAT, x1, x2, EV, left, right, w, fma=True)
    assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
    assert np.array_equal(sc.cpu().numpy(), fsc) and int(s.item()) == finc and fsc.sum() > 0


def test_nodes64_full_size_windows(ctx, oracle):
    """configs[3]'s per-GPU shard as the bench times it: 64 independent nodes
    x 2^20 f64 sites in two 32-node batched launches.  A 4096-site window of
    every node is checked bit for bit against the oracle on that window, and
    every node's scaler sum equals the sum of its scaler bytes (full size)."""
    import torch

    n, nn = 1 << 20, 64
    g = torch.Generator(device="cuda")
    g.manual_seed(64)
    EV = torch.rand(16, dtype=torch.float64, device="cuda", generator=g)
    wgt = torch.randint(0, 4, (n,), dtype=torch.int32, device="cuda", generator=g)
    sums = torch.full((nn,), -1, dtype=torch.int64, device="cuda")
    nodes = []
    for j in range(nn):
        x1 = torch.rand(16 * n, dtype=torch.float64, device="cuda", generator=g)
        x1.view(-1, 16)[j % 4::4] *= 1e-12
        nodes.append(dict(x1=x1, x2=torch.rand(16 * n, dtype=torch.float64, device="cuda", generator=g),
                          x3=torch.empty(16 * n, dtype=torch.float64, device="cuda"),
                          left=torch.rand(64, dtype=torch.float64, device="cuda", generator=g),
                          right=torch.rand(64, dtype=torch.float64, device="cuda", generator=g),
                          scaler=torch.empty(n, dtype=torch.uint8, device="cuda"),
                          scaler_sum=sums[j:j + 1]))
    ctx.plf_batch_dev(nodes[:32], EV, n, wgt)
    ctx.plf_batch_dev(nodes[32:], EV, n, wgt)
    torch.cuda.synchronize()
    h = lambda x: x.cpu().numpy()  # noqa: E731
    for j, nd in enumerate(nodes):
        lo = (j * 12289) % (n - 4096)
        sl = slice(16 * lo, 16 * (lo + 4096))
        e3, esc, einc = oracle.plf(h(nd["x1"][sl]), h(nd["x2"][sl]), h(EV), h(nd["left"]),
                                   h(nd["right"]), h(wgt[lo:lo + 4096]))
        assert np.array_equal(bits(h(nd["x3"][sl])), bits(e3)), j
        assert np.array_equal(h(nd["scaler"][lo:lo + 4096]), esc), j
        full = int((nd["scaler"].to(torch.int64) * wgt.to(torch.int64)).sum().item())
        assert int(sums[j].item()) == full, j
        assert int(nd["scaler"].sum().item()) >= n // 4
    del nodes
    torch.cuda.empty_cache()


def test_binding_rejects_host_or_mistyped_tensors(ctx):
    """The Python binding checks every tensor a kernel would read or write
    (the C ABI cannot see sizes or devices): host tensors, wrong dtypes and
    short buffers raise PlfxError before any launch."""
    import plfx
    import torch

    n = 64
    x = torch.zeros(16 * n, dtype=torch.float64, device="cuda")
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    bad_root = [
        dict(x=x.cpu(), out=out),                                      # host CLV
        dict(x=x.float()[: 8 * n], out=out),                            # short CLV
        dict(x=x, out=out.cpu()),                                       # host output
        dict(x=x, out=out, wgt=torch.ones(n, dtype=torch.int64, device="cuda")),
        dict(x=x, out=out, scaler_sums=torch.zeros(1, dtype=torch.int32, device="cuda")),
        dict(x=x, out=out, site_lnl=torch.zeros(n - 1, dtype=torch.float64, device="cuda")),
        dict(x=x, out=out, freq=torch.full((4,), 0.25, dtype=torch.float64)),
    ]
    for kw in bad_root:
        with pytest.raises(plfx.PlfxError):
            ctx.root_lnl(kw.pop("x"), n, kw.pop("out"), **kw)
    sc = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    for args in ((sc.cpu(), None, s), (sc, None, s.cpu()), (sc[: n - 1], None, s),
                 (sc, torch.ones(n, dtype=torch.int32), s)):
        with pytest.raises(plfx.PlfxError):
            ctx.scaler_sum(*args, n=n)
    e = torch.zeros(4 + 32, dtype=torch.float64, device="cuda")
    r = torch.ones(4, dtype=torch.float64, device="cuda")
    b = torch.ones(3, dtype=torch.float64, device="cuda")
    pm = torch.zeros(3 * 4 * 16, dtype=torch.float64, device="cuda")
    for args in ((e.cpu(), r, b, pm), (e, r, b, pm.cpu()), (e, r.float(), b, pm)):
        with pytest.raises(plfx.PlfxError):
            ctx.pmatrix(*args)
    # the valid forms still run
    ctx.scaler_sum(sc, None, s, n=n)
    torch.cuda.synchronize()
    assert int(s.item()) == 0


def _kernel_nodes(g):
    """Kernel nodes of a captured torch graph (made with keep_graph=True)."""
    import ctypes

    hip = _hip()
    graph = ctypes.c_void_p(int(g.raw_cuda_graph()))
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
    k = 0
    for nd in nodes:
        t = ctypes.c_int(-1)
        assert hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t)) == 0
        k += t.value == 0  # hipGraphNodeTypeKernel
    return k


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_tiptip_tables_on_a_first_call_inside_capture(oracle, dtype):
    """the tip/tip combination tables come with the
    workspace, so the FIRST call of a fresh context on a fresh stream, made
    inside a graph capture, takes the table path (2 kernels: the 576 code-pair
    tables, then the per-site gather) -- no allocation, no wait on the
    caller's stream.  Replays are bit-exact against the oracle."""
    import plfx
    import torch

    S, n = 20, 3001
    rng = np.random.default_rng(5)
    EV = (rng.random(S * S) - 0.25).astype(dtype)
    left = (rng.random(4 * S * S) * 1e-11).astype(dtype)
    right = rng.random(4 * S * S).astype(dtype)
    w = rng.integers(1, 5, n).astype(np.int32)
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1, e2 = oracle.expand_protein_tips(c1, dtype), oracle.expand_protein_tips(c2, dtype)
    f3, fsc, finc = oracle.plf_generic(S, 4, e1, e2, EV, left, right, w, fma=True)
    assert 0 < fsc.sum() < n
    t = [dev(a) for a in (c1, c2, EV, left, right, w)]
    x3 = torch.empty(4 * S * n, dtype=t[2].dtype, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    with plfx.Context(0) as c:
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=st):
            c.plf_tips_dev(x3, t[2], n, t[3], t[4], tip1=t[0], tip2=t[1], wgt=t[5], scaler=sc,
                           scaler_sum=s, states=S, fma=True, stream=st)
        assert _kernel_nodes(g) == 2
        g.instantiate()
        for _ in range(2):
            x3.zero_()
            s.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
            assert np.array_equal(sc.cpu().numpy(), fsc) and int(s.item()) == finc
        del g


def test_graph_kernel_launches_names_the_dispatch(ctx, oracle):
    """bench.graph_kernel_launches reads a captured graph's kernel nodes: the
    headline node call is one plf_dna_f64_pair_kernel dispatch of 256-thread
    workgroups over the co-resident grid -- what bench.py checks a PMC
    record's launch shapes against."""
    import sys

    import torch

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import bench
    from plfx import codeobj

    n = 1 << 16
    d = oracle.gen_hostmem(n, np.float64, 55)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    o3 = torch.empty_like(t["x1"])
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s, stream=st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=st):
        for _ in range(3):
            ctx.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s, stream=st)
    ls = bench.graph_kernel_launches(g)
    assert len(ls) == 3 and all(nm and codeobj._named(nm, "plf_dna_f64_pair_kernel") for nm, _, _ in ls)
    assert {w for _, _, w in ls} == {256} and len({gsz for _, gsz, _ in ls}) == 1
    ok, _ = bench.launch_check({"plf_dna_f64_pair_kernel": [[ls[0][1], 256]]}, ls)
    assert ok
    del g


def test_x3_partial_overlap_rejected(ctx):
    """a parent CLV sharing ANY byte with a child is
    refused (PLFX_ERR_INVALID) on every device entry point -- not only
    x3 == x1 -- while an adjacent, non-overlapping x3 is accepted."""
    import plfx
    import torch

    n = 1000
    for dt, V, states in ((torch.float64, 16, 4), (torch.float32, 16, 4), (torch.float64, 80, 20),
                          (torch.float32, 80, 20)):
        buf = torch.rand(V * (3 * n + 8), dtype=dt, device="cuda")
        x1, x2 = buf[:V * n], buf[V * n:2 * V * n]
        EV, P = torch.rand(states * states, dtype=dt, device="cuda"), torch.rand(4 * states * states, dtype=dt, device="cuda")
        step = 16 // buf.element_size()  # the smallest 16-B-aligned shift
        for x3 in (buf[step:step + V * n], buf[V * n - step:2 * V * n - step],   # into x1's tail
                   buf[2 * V * n - V * n // 2:3 * V * n - V * n // 2]):          # half into x2
            with pytest.raises(plfx.PlfxError) as ei:
                ctx.plf_dev_gen(x1, x2, x3, EV, P, P, states, n=n)
            assert ei.value.code == plfx.ERR_INVALID and "overlap" in str(ei.value)
            with pytest.raises(plfx.PlfxError) as ei:
                ctx.plf_batch_dev([dict(x1=x1, x2=x2, x3=x3, left=P, right=P)] * 2, EV, n, states=states)
            assert ei.value.code == plfx.ERR_INVALID and "overlap" in str(ei.value)
        ctx.plf_dev_gen(x1, x2, buf[2 * V * n:3 * V * n], EV, P, P, states, n=n)  # adjacent: fine
        if states == 4:
            x3 = buf[step:step + V * n]
            with pytest.raises(plfx.PlfxError) as ei:
                ctx.plf_dev(x1, x2, x3, EV, P, P, n=n)
            assert ei.value.code == plfx.ERR_INVALID
            # a coded tip child (one byte per site) inside the parent's bytes
            codes = buf[2 * V * n:3 * V * n].view(torch.uint8)[64:64 + n]
            with pytest.raises(plfx.PlfxError) as ei:
                ctx.plf_tips_dev(buf[2 * V * n:3 * V * n], EV, n, P, P, tip1=codes, x2=x2)
            assert ei.value.code == plfx.ERR_INVALID
    torch.cuda.synchronize()


def test_destroy_waits_for_its_streams_not_the_device(oracle):
    """plfx_ctx_destroy after the caller released its streams waits for the
    context's own work only, not for the whole device -- a long kernel on an
    unrelated stream is still running when close() returns; with a stream
    still holding a workspace (the handle may be dead, so it is
    never used) close() waits for the device instead, and that stream's work
    is complete afterwards."""
    import plfx
    import torch

    n = 1 << 18
    d = oracle.gen_hostmem(n, np.float64, 50)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    _, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    other, mine = torch.cuda.Stream(), torch.cuda.Stream()
    o3 = torch.empty_like(t["x1"])
    # calibrate torch's spin kernel
    t0 = time.perf_counter()
    torch.cuda._sleep(50_000_000)
    torch.cuda.synchronize()
    rate = 50_000_000 / max(time.perf_counter() - t0, 1e-4)
    # explicit: the caller releases `mine`; tracked: a torch stream, which
    # Context.close() releases itself; raw: an integer handle,
    # never remembered, so the workspace is still held at destroy
    for mode in ("explicit", "tracked", "raw"):
        s = torch.zeros(4, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        c = plfx.Context(0)
        for i in range(4):
            c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s[i:i + 1],
                      stream=mine.cuda_stream if mode == "raw" else mine)
        if mode == "explicit":
            c.release_stream(mine)
        with torch.cuda.stream(other):  # keep `other` busy for ~1.5 s
            torch.cuda._sleep(int(1.5 * rate))
            busy = torch.cuda.Event()
            busy.record(other)
        t0 = time.perf_counter()
        c.close()
        dt = time.perf_counter() - t0
        if mode != "raw":
            assert not busy.query(), f"close() waited for an unrelated stream ({mode})"
            assert dt < 0.5
        else:
            assert busy.query(), "close() with a held workspace must wait for the device"
        assert s.tolist() == [einc] * 4  # mine's launches were complete
        torch.cuda.synchronize()


def test_destroy_after_the_callers_stream_is_gone(oracle):
    """a stream that still holds a workspace may be
    destroyed by its owner before the context is (e.g. a Context collected at
    interpreter exit).  plfx_ctx_destroy never touches the dead handle (it
    waits for the device instead): the close returns, the sums of the
    stream's launches are complete, and a new context on the same device
    works."""
    import plfx
    import torch

    n = 1 << 18
    d = oracle.gen_hostmem(n, np.float64, 53)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    _, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    o3 = torch.empty_like(t["x1"])
    s = torch.zeros(6, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    c = plfx.Context(0)
    hs = _new_streams(3)
    for i, h in enumerate(hs):  # every stream takes a workspace, none is released
        for j in range(2):
            c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None,
                      s[2 * i + j:2 * i + j + 1], stream=h)
    _destroy_streams(hs)  # owner destroys them while their work may still run
    c.close()
    assert s.tolist() == [einc] * 6
    with plfx.Context(0) as c2:
        s2 = torch.zeros(1, dtype=torch.int64, device="cuda")
        c2.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None, s2)
        torch.cuda.synchronize()
        assert int(s2.item()) == einc


# the refused first capture ends with an empty graph, which torch warns about
@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lazy_tables_context(oracle, dtype):
    """plfx_ctx_create_ex(PLFX_CTX_LAZY_TABLES) skips the ~95 MB of
    protein tip/tip tables at creation (DNA-only users).  DNA works as
    before; a stream's FIRST tip/tip protein call inside a capture is refused
    with PLFX_ERR_INVALID (its tables would be allocated then); the same call
    outside a capture allocates them and is bit-exact, and later captures on
    that stream work."""
    import plfx
    import torch

    free0 = torch.cuda.mem_get_info()[0]
    S, n = 20, 3001
    rng = np.random.default_rng(9)
    EV = (rng.random(S * S) - 0.25).astype(dtype)
    left = (rng.random(4 * S * S) * 1e-11).astype(dtype)
    right = rng.random(4 * S * S).astype(dtype)
    w = rng.integers(1, 5, n).astype(np.int32)
    c1, c2 = oracle.random_protein_codes(rng, n, 0.3), oracle.random_protein_codes(rng, n, 0.3)
    e1, e2 = oracle.expand_protein_tips(c1, dtype), oracle.expand_protein_tips(c2, dtype)
    f3, fsc, finc = oracle.plf_generic(S, 4, e1, e2, EV, left, right, w, fma=True)
    t = [dev(a) for a in (c1, c2, EV, left, right, w)]
    x3 = torch.empty(4 * S * n, dtype=t[2].dtype, device="cuda")
    sc = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    with plfx.Context(0, lazy_tables=True) as c:
        assert free0 - torch.cuda.mem_get_info()[0] < 64 << 20  # no 95-MB table pool
        d = oracle.gen_hostmem(4099, dtype, 54)
        x = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
        e3, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
        o3, s0 = torch.empty_like(x["x1"]), torch.zeros(1, dtype=torch.int64, device="cuda")
        c.plf_dev(x["x1"], x["x2"], o3, x["EV"], x["left"], x["right"], x["wgt"], None, s0, stream=st)
        st.synchronize()
        assert np.array_equal(bits(o3.cpu().numpy()), bits(e3)) and int(s0.item()) == einc

        def call():
            c.plf_tips_dev(x3, t[2], n, t[3], t[4], tip1=t[0], tip2=t[1], wgt=t[5], scaler=sc,
                           scaler_sum=s, states=S, fma=True, stream=st)

        g = torch.cuda.CUDAGraph()
        with pytest.raises(plfx.PlfxError) as ei:
            with torch.cuda.graph(g, stream=st):
                call()
        assert ei.value.code == plfx.ERR_INVALID and "LAZY_TABLES" in str(ei.value)
        del g
        torch.cuda.synchronize()
        call()  # outside a capture: allocates this stream's tables
        st.synchronize()
        assert np.array_equal(bits(x3.cpu().numpy()), bits(f3))
        assert np.array_equal(sc.cpu().numpy(), fsc) and int(s.item()) == finc
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            call()
        x3.zero_()
        s.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(bits(x3.cpu().numpy()), bits(f3)) and int(s.item()) == finc
        del g


def test_release_after_capture_retires_the_workspace(oracle):
    """releasing a stream whose workspace a graph was
    captured through must not hand that workspace to another stream -- the
    graph's replays keep using its self-resetting sum words.  Capture on A,
    release A, then replay the graph on A while stream B makes sum-producing
    calls of its own: every sum exact.  Releasing a stream while it is being
    captured is refused."""
    import plfx
    import torch

    n = 1 << 18
    d = oracle.gen_hostmem(n, np.float64, 51)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    _, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    A, B = torch.cuda.Stream(), torch.cuda.Stream()
    oa, ob = torch.empty_like(t["x1"]), torch.empty_like(t["x1"])
    sa = torch.zeros(1, dtype=torch.int64, device="cuda")
    sb = torch.zeros(16, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with plfx.Context(0) as c:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=A):
            c.plf_dev(t["x1"], t["x2"], oa, t["EV"], t["left"], t["right"], t["wgt"], None, sa, stream=A)
            with pytest.raises(plfx.PlfxError) as ei:
                c.release_stream(A)
            assert ei.value.code == plfx.ERR_INVALID
        c.release_stream(A)  # retires A's workspace: the graph still uses it
        torch.cuda.synchronize()
        with torch.cuda.stream(A):
            for _ in range(8):
                g.replay()
        for i in range(16):  # B's first call takes a fresh pool entry
            c.plf_dev(t["x1"], t["x2"], ob, t["EV"], t["left"], t["right"], t["wgt"], None, sb[i:i + 1],
                      stream=B)
        torch.cuda.synchronize()
        assert int(sa.item()) == einc
        assert sb.tolist() == [einc] * 16
        c.release_stream(B)
        del g


def test_exited_threads_per_thread_workspaces_are_reclaimed(oracle):
    """a thread that used hipStreamPerThread and exits without
    releasing its workspace must not use up the context: PLFX_MAX_STREAMS + 6
    short-lived threads, one after another, each making one sum-producing
    call on its per-thread stream and exiting, all succeed with exact sums
    (the exited threads' entries are retired and reclaimed)."""
    import threading

    import plfx
    import torch

    n = 4099
    d = oracle.gen_hostmem(n, np.float64, 52)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    _, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    k = plfx.MAX_STREAMS + 6
    sums = torch.zeros(k, dtype=torch.int64, device="cuda")
    o3 = torch.empty_like(t["x1"])
    torch.cuda.synchronize()
    errs = []
    with plfx.Context(0) as c:
        def worker(i):
            try:
                c.plf_dev(t["x1"], t["x2"], o3, t["EV"], t["left"], t["right"], t["wgt"], None,
                          sums[i:i + 1], stream=plfx.STREAM_PER_THREAD)
                torch.cuda.current_stream().synchronize()
                hip = _hip()
                assert hip.hipStreamSynchronize(ctypes_stream_per_thread()) == 0
            except Exception as e:  # reported on the main thread
                errs.append(e)

        for i in range(k):
            th = threading.Thread(target=worker, args=(i,))
            th.start()
            th.join(timeout=60)
    assert not errs, errs[:3]
    torch.cuda.synchronize()
    assert sums.tolist() == [einc] * k


def ctypes_stream_per_thread():
    import ctypes

    import plfx

    return ctypes.c_void_p(plfx.STREAM_PER_THREAD)


def test_bound_launcher_keeps_its_tensors_alive(ctx, oracle):
    """bind_plf_dev / bind_plf_batch_dev launchers hold their tensors: with the
    caller's names gone and torch's cache emptied (what torch.cuda.graph does at
    capture start), the memory stays allocated -- checked BEFORE any launch --
    and the launcher still computes the right result."""
    import gc

    import torch

    n = 4099
    d = oracle.gen_hostmem(n, np.float64, 91)
    e3, _, einc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    torch.cuda.synchronize()
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    x3 = torch.empty_like(t["x1"])
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    run = ctx.bind_plf_dev(t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"], t["wgt"], None, s)
    nodes = [dict(x1=t["x1"], x2=t["x2"], x3=torch.empty_like(t["x1"]), left=t["left"], right=t["right"],
                  scaler=None, scaler_sum=torch.zeros(1, dtype=torch.int64, device="cuda"))]
    runb = ctx.bind_plf_batch_dev(nodes, t["EV"], n, t["wgt"])
    torch.cuda.synchronize()
    gc.collect()  # earlier tests' garbage first, so the comparison below sees only ours
    held = torch.cuda.memory_allocated()
    del t, x3, s, nodes
    gc.collect()
    torch.cuda.empty_cache()
    assert torch.cuda.memory_allocated() == held  # nothing of the launchers' was freed
    s = run.tensors[8]
    s.zero_()
    run()
    runb()
    torch.cuda.synchronize()
    assert np.array_equal(bits(run.tensors[2].cpu().numpy()), bits(e3)) and int(s.item()) == einc
    nb = runb.tensors[0][0]
    assert np.array_equal(bits(nb["x3"].cpu().numpy()), bits(e3)) and int(nb["scaler_sum"].item()) == einc


def test_bound_launcher_after_close_raises(oracle):
    """A launcher carries its context's handle: once the context is closed,
    using it raises PlfxError instead of passing a freed handle to the C ABI."""
    import plfx
    import torch

    n = 257
    d = oracle.gen_hostmem(n, np.float64, 92)
    t = {k: dev(d[k]) for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    c = plfx.Context(0)
    run = c.bind_plf_dev(t["x1"], t["x2"], torch.empty_like(t["x1"]), t["EV"], t["left"], t["right"],
                         t["wgt"])
    nodes = [dict(x1=t["x1"], x2=t["x2"], x3=torch.empty_like(t["x1"]), left=t["left"], right=t["right"])]
    runb = c.bind_plf_batch_dev(nodes, t["EV"], n, t["wgt"])
    run()
    runb()
    torch.cuda.synchronize()
    c.close()
    for r in (run, runb):
        with pytest.raises(plfx.PlfxError):
            r()


def test_context_releases_its_torch_streams_on_close(oracle):
    """a Context remembers the torch streams it ran on and
    releases their workspaces at close() (plfx_ctx_release_stream), so
    destroy does not fall back to a device-wide wait; raw integer handles are
    not remembered; release_stream() forgets the stream."""
    import torch

    import plfx

    n = 4099
    d = oracle.gen_hostmem(n, np.float64, 3)
    t = {k: torch.from_numpy(d[k]).cuda() for k in ("x1", "x2", "EV", "left", "right", "wgt")}
    x3 = torch.empty_like(t["x1"])
    s = torch.zeros(1, dtype=torch.int64, device="cuda")
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    c = plfx.Context(0)
    args = (t["x1"], t["x2"], x3, t["EV"], t["left"], t["right"], t["wgt"], None, s)
    c.plf_dev(*args, stream=a)
    c.plf_dev(*args, stream=b)
    c.plf_dev(*args, stream=b.cuda_stream)   # raw handle: not remembered
    c.plf_dev(*args)                          # torch's current stream
    assert set(c._used) == {a.cuda_stream, b.cuda_stream, torch.cuda.current_stream().cuda_stream}
    c.release_stream(a)
    assert a.cuda_stream not in c._used
    torch.cuda.synchronize()
    c.close()
    assert c._used == {} and c.h is None
    e3, _, _ = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], d["wgt"])
    assert np.array_equal(x3.cpu().numpy().view(np.uint64), e3.view(np.uint64))
