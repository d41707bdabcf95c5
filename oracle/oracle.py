"""CPU oracle for the PLF hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product (``libplfx.so``, its HIP kernels, the C++ host driver and the
``plfx`` Python binding) never imports, links or calls anything here.

Contents
--------
* ctypes bindings to ``liboracle.so`` (``plf_oracle.c``): the clean-room
  restatement of ``plf()`` (/root/reference/app/src/plf.cpp:8-68) in float and
  double, a generic S-state/C-category form, the host_mem input protocol
  (/root/reference/app/src/host_mem.cpp:179-209) and the scaler reduction
  (host_mem.cpp:384-388).
* ctypes bindings to the reference's own ``plf()`` built into ``oracle/_ref``
  from /root/reference/app/src/plf.cpp (oracle/Makefile), used to pin the
  restatement, and ``ref_traverse``: a tree sweep as the composition of the
  reference's own plf() calls, one per inner node in post-order, which pins
  the traversal/fused-pass results of BASELINE configs[2]/[3].
* ``testbench_*``: the instance sizing/partition arithmetic of
  ``testbench_info`` (/root/reference/app/src/include.h:150-266).
* ``pack_instance``: the per-instance input buffers of host_mem.cpp:221-243.
* ``mm2s_lane_streams`` / ``s2mm``: the PL data movers
  (hls/src/mm2sleft_memDNAwindowComb.cpp:16-100, mm2sright_*,
  mm2sleft_memDNAwindowSep.cpp:16-95, mm2sright_memDNAwindowSep.cpp:16-88,
  mm2sleft_memDNAstreamComb.cpp:16-116, transpose.cpp:6-24,
  s2mm_memDNAwindowComb.cpp:20-101), restated over numpy so that the
  AIE test vectors in aie/data pin the packing.
* ``parse_aie_kat``: reads the reference's AIE golden vectors
  (aie/data/golden{0..3}.txt and their stimuli).

Parity status: the float path is pinned (reference binary + AIE goldens +
committed fixtures); double by the reference source's double instantiation;
4-state tree sweeps (dense and state-coded tips) by the composition of the
reference's plf() calls (tests/golden/tree64.npz, ref_traverse); the S-state
(protein) loop on the embedded 4-state sub-space (embed_dna_*: a DNA problem
in states 0..3 of 20 must reproduce the reference's plf() bit for bit), and
the fused-multiply-add form (PLFX_FMA) by the reference source compiled with
FMA contraction (oracle/_ref/libplfref{,_f64}_fma.so).  The protein loop
beyond that sub-space (chains longer than 4 terms) and the root lnL are
extensions the reference does not have: parity unpinned beyond being the same
loop as the pinned path.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"
REF_O0 = ORACLE_DIR / "_ref" / "libplfref_O0.so"
REF_O3 = ORACLE_DIR / "_ref" / "libplfref_O3.so"

TWO_TO_32 = 4294967296.0
MINLIKELIHOOD = 1.0 / TWO_TO_32
SEED = 20250117

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")

_lib = None
_refs: dict = {}


def build():
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def _gen_omp_argtypes(L, sfx, fp):
    f = getattr(L, f"plfo_plf_gen_omp_{sfx}")
    f.argtypes = [C.c_int, C.c_int, C.c_int, fp, fp, fp, fp, C.c_longlong, fp, fp,
                  C.c_void_p, C.POINTER(C.c_longlong), C.c_void_p, C.c_int]
    f.restype = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        for sfx, fp in (("f32", _f32p), ("f64", _f64p)):
            f = getattr(L, f"plfo_plf_{sfx}")
            f.argtypes = [fp, fp, fp, fp, C.c_longlong, fp, fp, C.c_void_p,
                          C.POINTER(C.c_int), C.c_void_p]
            f.restype = None
            f = getattr(L, f"plfo_plf_{sfx}_omp")
            f.argtypes = [fp, fp, fp, fp, C.c_longlong, fp, fp, C.c_void_p,
                          C.POINTER(C.c_int), C.c_void_p, C.c_int]
            f.restype = None
            f = getattr(L, f"plfo_plf_gen_{sfx}")
            f.argtypes = [C.c_int, C.c_int, fp, fp, fp, fp, C.c_longlong, fp, fp,
                          C.c_void_p, C.POINTER(C.c_longlong), C.c_void_p]
            f.restype = None
            f = getattr(L, f"plfo_plf_gen_fma_{sfx}")
            f.argtypes = [C.c_int, C.c_int, fp, fp, fp, fp, C.c_longlong, fp, fp,
                          C.c_void_p, C.POINTER(C.c_longlong), C.c_void_p]
            f.restype = None
            _gen_omp_argtypes(L, sfx, fp)
            f = getattr(L, f"plfo_gen_hostmem_{sfx}")
            f.argtypes = [C.c_uint32, C.c_longlong, fp, fp, fp, fp, fp, C.c_void_p]
            f.restype = None
        for sfx in ("f32", "f64"):
            f = getattr(L, f"plfo_traverse_{sfx}")
            f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                          C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
            f.restype = None
            f = getattr(L, f"plfo_root_lnl_{sfx}")
            f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p,
                          C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
            f.restype = C.c_double
        L.plfo_scaler_sum.argtypes = [_u8p, C.c_void_p, C.c_longlong]
        L.plfo_scaler_sum.restype = C.c_longlong
        L.plfo_mt_draws.argtypes = [C.c_uint32, C.c_longlong, C.c_void_p, C.c_void_p]
        L.plfo_mt_draws.restype = None
        _lib = L
    return _lib


def native_lib():
    """The restatement built on THIS machine at -O3 -march=native
    -ffp-contract=off (oracle/Makefile `native`), for the CPU-baseline
    variant; None when it cannot be built here."""
    global _native
    if _native is None:
        import subprocess

        p = ORACLE_DIR / "_native" / "liboracle_native.so"
        try:
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR), "native"], check=True,
                           capture_output=True, timeout=120)
        except (OSError, subprocess.SubprocessError):
            _native = False
            return None
        L = C.CDLL(str(p))
        for sfx, fp in (("f32", _f32p), ("f64", _f64p)):
            f = getattr(L, f"plfo_plf_{sfx}")
            f.argtypes = [fp, fp, fp, fp, C.c_longlong, fp, fp, C.c_void_p,
                          C.POINTER(C.c_int), C.c_void_p]
            f.restype = None
            f = getattr(L, f"plfo_plf_{sfx}_omp")
            f.argtypes = [fp, fp, fp, fp, C.c_longlong, fp, fp, C.c_void_p,
                          C.POINTER(C.c_int), C.c_void_p, C.c_int]
            f.restype = None
            for name in (f"plfo_plf_gen_{sfx}", f"plfo_plf_gen_fma_{sfx}"):
                f = getattr(L, name)
                f.argtypes = [C.c_int, C.c_int, fp, fp, fp, fp, C.c_longlong, fp, fp,
                              C.c_void_p, C.POINTER(C.c_longlong), C.c_void_p]
                f.restype = None
            _gen_omp_argtypes(L, sfx, fp)
        _native = L
    return _native or None


_native = None


def ref_lib(opt: str = "O0"):
    """The reference plf() itself (oracle/_ref), or None if it was not built.
    opt: "O0" (its own host flags), "O3", "O3v4" (-O3 -march=x86-64-v4), "fma"
    (-O3 -march=x86-64-v3 -ffp-contract=fast: every multiply-add fused)."""
    if opt not in _refs:
        p = {"O0": REF_O0, "O3": REF_O3}.get(opt, ORACLE_DIR / "_ref" / f"libplfref_{opt}.so")
        if not p.exists():
            _refs[opt] = None
        else:
            L = C.CDLL(str(p))
            L.plfref_plf.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, _f32p,
                                     _f32p, _i32p]
            L.plfref_plf.restype = C.c_int
            _refs[opt] = L
    return _refs[opt]


def ref_lib_f64(opt: str = "O0"):
    """The reference plf()'s double instantiation (oracle/ref_shim_f64.cpp:
    the unmodified plf.cpp compiled with float spelled double), or None."""
    key = "f64_" + opt
    if key not in _refs:
        p = ORACLE_DIR / "_ref" / f"libplfref_f64_{opt}.so"
        if not p.exists():
            _refs[key] = None
        else:
            L = C.CDLL(str(p))
            f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
            L.plfref_plf_f64.argtypes = [f64p, f64p, f64p, f64p, C.c_int, f64p, f64p, _i32p]
            L.plfref_plf_f64.restype = C.c_int
            _refs[key] = L
    return _refs[key]


def ref_plf_f64(x1, x2, EV, left, right, wgt, opt="O0"):
    """(x3, scalerIncrement) from the reference's own loop in double, or None
    when oracle/_ref holds no f64 build."""
    L = ref_lib_f64(opt)
    if L is None:
        return None
    c = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    a1, a2 = c(x1), c(x2)
    n = a1.size // 16
    x3 = np.empty(16 * n, np.float64)
    inc = L.plfref_plf_f64(a1, a2, x3, c(EV), n, c(left), c(right), np.ascontiguousarray(wgt, np.int32))
    return x3, int(inc)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _sfx(dtype):
    return "f32" if np.dtype(dtype) == np.float32 else "f64"


# --------------------------------------------------------------------------
# plf() and friends
# --------------------------------------------------------------------------
def plf(x1, x2, EV, left, right, wgt=None, n=None, threads=0, out=None, L=None):
    """Restated plf(): returns (x3, scaler_bytes, scalerIncrement).

    threads > 0 uses the OpenMP variant (identical results); `out` may supply
    preallocated (x3, scaler) arrays; L another build of the same source
    (native_lib())."""
    dt = x1.dtype
    if n is None:
        n = x1.size // 16
    if out is not None:
        x3, sc = out
    else:
        x3 = np.empty(n * 16, dtype=dt)
        sc = np.empty(n, dtype=np.uint8)
    inc = C.c_int(0)
    L = L or lib()
    if wgt is not None:
        wgt = np.ascontiguousarray(wgt, dtype=np.int32)
    if threads > 0:
        getattr(L, f"plfo_plf_{_sfx(dt)}_omp")(x1, x2, x3, EV, n, left, right,
                                              _ptr(wgt), C.byref(inc), _ptr(sc), threads)
    else:
        getattr(L, f"plfo_plf_{_sfx(dt)}")(x1, x2, x3, EV, n, left, right,
                                          _ptr(wgt), C.byref(inc), _ptr(sc))
    return x3, sc, inc.value


def plf_generic(S, Ccat, x1, x2, EV, left, right, wgt=None, fma=False, threads=0, L=None):
    """Generic S-state / C-category restatement (protein S=20): unpinned
    extension; identical to plf() for S=C=4.  fma=True: every multiply-add
    fused in the same order (the PLFX_FMA mode).  threads > 0: the OpenMP
    variant (identical results); L another build of the same source
    (native_lib())."""
    dt = x1.dtype
    V = S * Ccat
    n = x1.size // V
    x3 = np.empty(n * V, dtype=dt)
    sc = np.empty(n, dtype=np.uint8)
    inc = C.c_longlong(0)
    if wgt is not None:
        wgt = np.ascontiguousarray(wgt, dtype=np.int32)
    L = L or lib()
    if threads > 0:
        getattr(L, f"plfo_plf_gen_omp_{_sfx(dt)}")(int(fma), S, Ccat, x1, x2, x3, EV, n, left, right,
                                                   _ptr(wgt), C.byref(inc), _ptr(sc), threads)
        return x3, sc, inc.value
    name = f"plfo_plf_gen_fma_{_sfx(dt)}" if fma else f"plfo_plf_gen_{_sfx(dt)}"
    getattr(L, name)(S, Ccat, x1, x2, x3, EV, n, left, right, _ptr(wgt), C.byref(inc), _ptr(sc))
    return x3, sc, inc.value


def traverse(S, Ccat, ops, clv, pmats, EV, n, wgt=None, want_scalers=False):
    """Sequential traversal (extension, unpinned): ops = int32 array (nops, 4)
    [parent, child1, child2, pmat]; clv = list of numpy CLVs (slots, written in
    place); pmats = flat array of 2*npmat matrices (C*S*S each).
    Returns (scaler_sums int64[nops], scalers list or None)."""
    ops = np.ascontiguousarray(ops, dtype=np.int32).reshape(-1, 4)
    nops = ops.shape[0]
    dt = clv[0].dtype
    ptrs = (C.c_void_p * len(clv))(*[a.ctypes.data_as(C.c_void_p) for a in clv])
    sums = np.zeros(nops, np.int64)
    scal = [np.zeros(n, np.uint8) for _ in range(nops)] if want_scalers else None
    sptr = (C.c_void_p * nops)(*[a.ctypes.data_as(C.c_void_p) for a in scal]) if scal else None
    w = None if wgt is None else np.ascontiguousarray(wgt, np.int32)
    getattr(lib(), f"plfo_traverse_{_sfx(dt)}")(S, Ccat, ops.ctypes.data_as(C.c_void_p), nops, ptrs,
                                               np.ascontiguousarray(pmats, dt).ctypes.data_as(C.c_void_p),
                                               np.ascontiguousarray(EV, dt).ctypes.data_as(C.c_void_p),
                                               n, _ptr(w), sptr, sums.ctypes.data_as(C.c_void_p))
    return sums, scal


def root_lnl(S, Ccat, x, n, catw=None, freq=None, wgt=None, scaler_sums=None, site=False):
    """Root log-likelihood (extension, unpinned):
    sum_i wgt_i log(sum_c catw_c sum_s freq_s x[i,c,s]) + sum(scaler_sums)*log(2^-32)."""
    dt = x.dtype
    sl = np.empty(n, np.float64) if site else None
    ss = None if scaler_sums is None else np.ascontiguousarray(scaler_sums, np.int64)
    cw = None if catw is None else np.ascontiguousarray(catw, np.float64)
    fr = None if freq is None else np.ascontiguousarray(freq, np.float64)
    w = None if wgt is None else np.ascontiguousarray(wgt, np.int32)
    v = getattr(lib(), f"plfo_root_lnl_{_sfx(dt)}")(S, Ccat, x.ctypes.data_as(C.c_void_p), n,
                                                    _ptr(cw), _ptr(fr), _ptr(w), _ptr(ss),
                                                    0 if ss is None else ss.size, _ptr(sl))
    return (v, sl) if site else v


def balanced_tree_ops(ntips):
    """Post-order ops of a balanced binary tree over `ntips` tips (power of 2):
    slots 0..ntips-1 are tips, inner nodes get slots ntips.. in post-order
    (level by level); op j uses P-matrix pair j.  Returns int32 (ntips-1, 4)."""
    ops = []
    level = list(range(ntips))
    nxt = ntips
    while len(level) > 1:
        new = []
        for i in range(0, len(level), 2):
            ops.append((nxt, level[i], level[i + 1], len(ops)))
            new.append(nxt)
            nxt += 1
        level = new
    return np.array(ops, np.int32)


TREE_GOLDEN_N = 257       # ragged: not a multiple of any kernel's trip
TREE_GOLDEN_SEED = 6464


TREE_GOLDEN_TIPS = ("dense", "coded", "mixed", "tipvec")


def tree_golden_case(dtype, coded, n=TREE_GOLDEN_N, seed=TREE_GOLDEN_SEED):
    """Inputs of the committed tree-sweep fixtures (tests/golden/tree64.npz):
    BASELINE configs[2]'s 64-taxon balanced tree at a small ragged site count,
    P and EV scaled by 0.25 so the deep levels underflow and the
    scaler path runs.  coded: False / "dense" (every tip a dense CLV), True /
    "coded" (every tip DNA state codes, 20 % ambiguous, expanded to the dense
    CLV plf() reads), "mixed" (tips 4j+1 and 4j+2 coded, the rest dense:
    tip/tip, tip/inner and inner/inner nodes) or "tipvec" (every tip coded,
    expanded through a caller tip-vector table of signed values, as eigen-
    coordinate tips are).  Returns dict(ops, tips (dense CLVs), codes (per tip:
    codes or None), tipvec (16 x 4 or None), pm, EV, wgt, n)."""
    mode = {False: "dense", True: "coded"}.get(coded, coded)
    dt = np.dtype(dtype)
    rng = np.random.default_rng(seed + TREE_GOLDEN_TIPS.index(mode))
    ops = balanced_tree_ops(64)
    is_coded = [mode in ("coded", "tipvec") or (mode == "mixed" and t % 4 in (1, 2)) for t in range(64)]
    codes = [random_tip_codes(rng, n, 0.2) if c else None for c in is_coded]
    dense = [None if c else rng.random(16 * n).astype(dt) for c in is_coded]
    tv = (rng.random(64) - 0.25).astype(dt) if mode == "tipvec" else None
    tips = [expand_tips(c, dt, tipvec=tv) if c is not None else d for c, d in zip(codes, dense)]
    pm = (rng.random(ops.shape[0] * 128) * 0.25).astype(dt)
    EV = (rng.random(16) * 0.25).astype(dt)
    wgt = rng.integers(1, 5, n).astype(np.int32)
    return dict(ops=ops, tips=tips, codes=codes, tipvec=tv, pm=pm, EV=EV, wgt=wgt, n=n)


def tree_case_digest(case):
    """sha256 over a tree case's input bytes (tips, P, EV, weights): a fixture
    is only compared when the inputs regenerate to the same bytes."""
    import hashlib

    h = hashlib.sha256()
    for t in case["tips"]:
        h.update(np.ascontiguousarray(t).tobytes())
    for k in ("pm", "EV", "wgt"):
        h.update(np.ascontiguousarray(case[k]).tobytes())
    return h.hexdigest()


def embed_dna_clv(x, S=20):
    """A 4-state CLV [site][cat][4] placed in states 0..3 of an S-state CLV
    [site][cat][S], every other value +0.0.  With P and EV embedded the same way
    (embed_dna_mats), plf()'s S-state loop adds only exact +0.0 terms to the
    4-state chains (x*0 = +0, v + +0 = v for every chain value plf() can hold)
    and tests 4*(S-4) extra +0 values (< 2^-32) in the scale test, so its
    states 0..3 reproduce the 4-state plf() bit for bit and states 4.. stay +0:
    the reference's own plf() pins the S-state kernels on this sub-space."""
    x = np.asarray(x)
    n = x.size // 16
    out = np.zeros((n, 4, S), x.dtype)
    out[:, :, :4] = x.reshape(n, 4, 4)
    return out.reshape(-1)


def embed_dna_mats(m, S=20):
    """4x4 matrices (DNA P pairs [cat][k][l] of 64 values, or EV of 16) -> S x S
    with the 4x4 block top-left, zeros elsewhere (same count of matrices)."""
    m = np.asarray(m)
    k = m.size // 16
    out = np.zeros((k, S, S), m.dtype)
    out[:, :4, :4] = m.reshape(k, 4, 4)
    return out.reshape(-1)


def embed_clv_blocks(xs, S=20):
    """CLVs of len(xs) <= S/4 4-state problems in states 4b..4b+3, rest +0.0."""
    n = xs[0].size // 16
    out = np.zeros((n, 4, S), xs[0].dtype)
    for b, x in enumerate(xs):
        out[:, :, 4 * b:4 * b + 4] = np.asarray(x).reshape(n, 4, 4)
    return out.reshape(-1)


def embed_mat_blocks(ms, S=20):
    """Matrices (P pairs of 64 or EV of 16 values each) of len(ms) problems as
    the diagonal 4x4 blocks of S x S matrices, zeros elsewhere."""
    k = np.asarray(ms[0]).size // 16
    out = np.zeros((k, S, S), np.asarray(ms[0]).dtype)
    for b, m in enumerate(ms):
        out[:, 4 * b:4 * b + 4, 4 * b:4 * b + 4] = np.asarray(m).reshape(k, 4, 4)
    return out.reshape(-1)


def extract_clv_blocks(xp, nblocks, S=20):
    """(the nblocks 4-state CLVs, whether every state past them is +0.0)."""
    xp = np.asarray(xp)
    n = xp.size // (4 * S)
    v = xp.reshape(n, 4, S)
    outs = [np.ascontiguousarray(v[:, :, 4 * b:4 * b + 4]).reshape(-1) for b in range(nblocks)]
    return outs, bool(not v[:, :, 4 * nblocks:].view(np.uint8).any())


def extract_dna_clv(xp, S=20):
    """Inverse of embed_dna_clv: (states 0..3 as a 4-state CLV, whether every
    other value is exactly +0.0)."""
    xp = np.asarray(xp)
    n = xp.size // (4 * S)
    v = xp.reshape(n, 4, S)
    rest = v[:, :, 4:]
    return np.ascontiguousarray(v[:, :, :4]).reshape(-1), bool(not rest.view(np.uint8).any())


def embedded_dna_tipvec(dtype, S=20):
    """Protein tip-vector table (PROT_CODES x S) whose rows 0..15 are the DNA
    state-code indicators (bit l of the code in state l, states 4.. zero): a
    DNA code c & 15 used as a protein code reads exactly the embedded DNA tip."""
    tv = np.zeros((PROT_CODES, S), dtype)
    for c in range(16):
        tv[c, :4] = [(c >> l) & 1 for l in range(4)]
    return tv.reshape(-1)


def clv_digest(a):
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def expand_tips(codes, dtype=np.float64, Ccat=4, tipvec=None):
    """Dense CLV of a tip stored as DNA state codes (bit s = state s possible,
    upper nibble ignored; the RAxML/PLL encoding): x[i][c][s] = (code_i >> s) & 1
    for every category c, or tipvec[code_i & 15][s] when a 16 x 4 tip-vector
    table is given.  This is the definition the GPU's tip path is checked
    against (plfx.h section 8): plf() on the expanded CLV."""
    codes = np.asarray(codes, np.uint8)
    if tipvec is None:
        rows = ((codes[:, None] >> np.arange(4, dtype=np.uint8)) & 1).astype(dtype)
    else:
        rows = np.asarray(tipvec, dtype).reshape(16, 4)[codes & 15]
    return np.ascontiguousarray(np.repeat(rows[:, None, :], Ccat, axis=1).reshape(-1))


PROT_CODES = 24


def protein_tip_table(dtype=np.float64, tipvec=None):
    """The protein tip-vector table (plfx.h section 8): PROT_CODES rows of 20
    states in ARNDCQEGHILKMFPSTWYV order -- 0..19 one state, 20 = B (N|D),
    21 = Z (Q|E), 22 = X, 23 = gap (all states) -- or the caller's table."""
    if tipvec is not None:
        return np.asarray(tipvec, dtype).reshape(PROT_CODES, 20)
    t = np.zeros((PROT_CODES, 20), dtype)
    t[np.arange(20), np.arange(20)] = 1
    t[20, [2, 3]] = 1
    t[21, [5, 6]] = 1
    t[22:] = 1
    return t


def expand_protein_tips(codes, dtype=np.float64, Ccat=4, tipvec=None):
    """Dense protein CLV of a tip stored as code indices (codes >= PROT_CODES
    read the last row): x[i][c][s] = table[code_i][s] for every category."""
    codes = np.minimum(np.asarray(codes, np.uint8), PROT_CODES - 1)
    rows = protein_tip_table(dtype, tipvec)[codes]
    return np.ascontiguousarray(np.repeat(rows[:, None, :], Ccat, axis=1).reshape(-1))


def random_protein_codes(rng, n, ambiguous=0.1):
    """Mostly single amino acids (0..19), a fraction of B/Z/X/gap and junk >= 24."""
    codes = rng.integers(0, 20, n).astype(np.uint8)
    amb = rng.random(n) < ambiguous
    codes[amb] = rng.integers(20, 256, int(amb.sum())).astype(np.uint8)
    return codes


def random_tip_codes(rng, n, ambiguous=0.1):
    """Tip codes: mostly unambiguous A/C/G/T (1, 2, 4, 8), a fraction of
    random bytes (ambiguity codes, gaps 15, code 0, junk in the upper nibble)."""
    codes = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, n)]
    amb = rng.random(n) < ambiguous
    codes[amb] = rng.integers(0, 256, int(amb.sum())).astype(np.uint8)
    return codes


def ref_plf(x1, x2, EV, left, right, wgt, opt="O0"):
    """Run the reference plf() (float only).  Returns (x3, scalerIncrement)."""
    L = ref_lib(opt)
    if L is None:
        raise FileNotFoundError("oracle/_ref was not built (no /root/reference here)")
    n = x1.size // 16
    x3 = np.zeros(n * 16, dtype=np.float32)
    inc = L.plfref_plf(x1.copy(), x2.copy(), x3, EV.copy(), n, left.copy(), right.copy(),
                       np.ascontiguousarray(wgt, dtype=np.int32).copy())
    return x3, inc


def _ref_call(dtype, opt="O0"):
    """The reference plf() entry of one dtype over raw contiguous arrays:
    f(x1, x2, x3, EV, n, left, right, wgt) -> scalerIncrement, or None.
    opt "fma": the build with every multiply-add contracted (oracle/Makefile)."""
    if np.dtype(dtype) == np.float32:
        L = ref_lib(opt)
        return None if L is None else L.plfref_plf
    L = ref_lib_f64(opt)
    return None if L is None else L.plfref_plf_f64


def ref_available(dtype=np.float32, opt="O0") -> bool:
    return _ref_call(dtype, opt) is not None


def ref_scaled_sites(f, x1, x2, EV, left, right, n):
    """Per-site scaler bytes of one reference plf() call (the reference returns
    only the weighted sum): each half of a site range is called with unit
    weights and split further only while its count is neither 0 nor its length,
    so sparse and dense scaling cost O(scaled · log n) calls, not n."""
    sc = np.zeros(n, np.uint8)
    V = x1.size // n
    ones = np.ones(n, np.int32)
    x3 = np.empty_like(x1)

    def count(lo, hi):
        return f(x1[V * lo:V * hi], x2[V * lo:V * hi], x3[V * lo:V * hi], EV, hi - lo, left, right,
                 ones[lo:hi])

    stack = [(0, n, count(0, n))] if n else []
    while stack:
        lo, hi, c = stack.pop()
        if c == 0:
            continue
        if c == hi - lo:
            sc[lo:hi] = 1
            continue
        mid = (lo + hi) // 2
        cl = count(lo, mid)
        stack.append((lo, mid, cl))
        stack.append((mid, hi, c - cl))
    return sc


def ref_traverse(ops, clv, pmats, EV, n, wgt=None, want_scalers=False, opt="O0"):
    """A traversal as the reference would run it: the UNMODIFIED reference
    plf() (/root/reference/app/src/plf.cpp:8-68, oracle/_ref; the f64 build is
    the same source with float spelled double) called once per op in op order
    -- parent = plf(child1, child2, P_left, P_right) -- exactly how a tree
    likelihood code calls it per inner node.  ops = int32
    (nops, 4) [parent, child1, child2, pmat]; clv = list of numpy CLVs (4-state,
    written in place); pmats = flat 2·npmat 4×4×4 matrices; wgt None = 1.
    Returns (scaler_sums int64[nops], scaler bytes per op or None).
    Raises FileNotFoundError when oracle/_ref holds no build for the dtype."""
    dt = clv[0].dtype
    f = _ref_call(dt, opt)
    if f is None:
        raise FileNotFoundError("oracle/_ref was not built (no /root/reference here)")
    ops = np.ascontiguousarray(ops, dtype=np.int32).reshape(-1, 4)
    pm = np.ascontiguousarray(pmats, dt)
    ev = np.ascontiguousarray(EV, dt)
    w = np.ones(n, np.int32) if wgt is None else np.ascontiguousarray(wgt, np.int32)
    sums = np.zeros(ops.shape[0], np.int64)
    scal = [] if want_scalers else None
    for j, (p, c1, c2, m) in enumerate(ops):
        left, right = pm[128 * m:128 * m + 64], pm[128 * m + 64:128 * m + 128]
        x1, x2 = clv[c1].copy(), clv[c2].copy()  # a parent may reuse a child's slot
        out = np.empty(16 * n, dt)
        sums[j] = f(x1, x2, out, ev, n, left, right, w) if n else 0
        clv[p][:] = out
        if want_scalers:
            scal.append(ref_scaled_sites(f, x1, x2, ev, left, right, n))
    return sums, scal


def scaler_sum(scaler, wgt=None):
    return lib().plfo_scaler_sum(np.ascontiguousarray(scaler, dtype=np.uint8),
                                 _ptr(None if wgt is None else np.ascontiguousarray(wgt, np.int32)),
                                 scaler.size)


def gen_hostmem(n, dtype=np.float32, seed=SEED):
    """host_mem.cpp:179-209 input protocol with a fixed seed (the reference uses
    std::random_device; Q8).  Returns dict(EV, left, right, x1, x2, wgt)."""
    dt = np.dtype(dtype)
    ev = np.empty(16, dt)
    left = np.empty(64, dt)
    right = np.empty(64, dt)
    x1 = np.empty(16 * n, dt)
    x2 = np.empty(16 * n, dt)
    wgt = np.empty(n, np.int32)
    getattr(lib(), f"plfo_gen_hostmem_{_sfx(dt)}")(seed, n, ev, left, right, x1, x2,
                                                   _ptr(wgt))
    return dict(EV=ev, left=left, right=right, x1=x1, x2=x2, wgt=wgt)


def mt_draws(seed, count):
    a = np.empty(count, np.uint32)
    d = np.empty(count, np.float64)
    lib().plfo_mt_draws(seed, count, _ptr(a), _ptr(d))
    return a, d


# --------------------------------------------------------------------------
# testbench_info sizing (include.h:150-266), COMBINED=0 / SEPARATE=1,
# STREAM=0 / WINDOW=1 as in include.h:20-21.
# --------------------------------------------------------------------------
COMBINED, SEPARATE = 0, 1
STREAM, WINDOW = 0, 1


class Testbench:
    def __init__(self, alignment_sites, parallel_instances=1, window_size=1024,
                 layout=SEPARATE, aie_type=WINDOW, plf_calls=1):
        self.alignment_sites = int(alignment_sites)
        self.parallel_instances = int(parallel_instances)
        self.window_size = int(window_size)
        self.input_layout = layout
        self.aie_type = aie_type
        self.plf_calls = plf_calls
        self.elements_per_alignment = 16

    def alignments_per_window(self):
        return self.window_size >> 4

    def alignments_per_instance(self, k=None):
        n0 = int(math.ceil(self.alignment_sites / self.parallel_instances))
        if k is None:
            return n0
        return n0 - (k == self.parallel_instances - 1) * self.alignments_padding()

    def alignments_padding(self):
        return self.alignments_per_instance() * self.parallel_instances - self.alignment_sites

    def alignmentelements_per_instance(self, k):
        return self.alignments_per_instance(k) * 16

    def num_windows_per_instance(self):
        apw = self.alignments_per_window()
        full = self.alignments_per_instance() // apw
        rem = self.alignments_per_instance() - full * apw
        return full + (rem > 0)

    def stream_padding(self):
        return self.alignment_sites & 1

    def elements_per_instance(self):
        if self.aie_type == STREAM:
            r = self.alignments_per_instance() + self.stream_padding()
        else:
            r = self.num_windows_per_instance() * self.alignments_per_window()
        return r * 16

    def header_left(self):
        return 5 * 16

    def header_right(self):
        return 4 * 16 if self.input_layout == SEPARATE else 5 * 16

    def instance_elements_left(self):
        return self.elements_per_instance() + self.header_left()

    def instance_elements_right(self):
        return self.elements_per_instance() + self.header_right()

    def instance_elements_out(self):
        return self.elements_per_instance()

    def instance_active_elements_left(self, k):
        return self.alignmentelements_per_instance(k) + self.header_left()

    def instance_active_elements_right(self, k):
        return self.alignmentelements_per_instance(k) + self.header_right()

    def instance_site_offset(self, k):
        # host_mem.cpp:229 / :290-291: offsets use instance 0's size
        return k * self.alignments_per_instance(0)


def pack_instance(tb: Testbench, k, EV, left, right, x1, x2, fill=0.0):
    """Per-instance input buffers of host_mem.cpp:221-243 (whole padded
    device buffers; the reference leaves the padded tail uninitialised, Q5:
    here it is `fill`)."""
    dt = x1.dtype
    L = np.full(tb.instance_elements_left(), fill, dtype=dt)
    R = np.full(tb.instance_elements_right(), fill, dtype=dt)
    off = tb.instance_site_offset(k) * 16
    cnt = tb.alignmentelements_per_instance(k)
    L[0:16] = EV
    L[16:80] = left
    L[80:80 + cnt] = x1[off:off + cnt]
    if tb.input_layout == COMBINED:
        R[0:16] = EV
        R[16:80] = right
        R[80:80 + cnt] = x2[off:off + cnt]
    else:
        R[0:64] = right
        R[64:64 + cnt] = x2[off:off + cnt]
    return L, R


def transpose4(word16):
    """transpose.cpp:6-24: element i*4+j -> j*4+i."""
    return np.asarray(word16).reshape(4, 4).T.reshape(16).copy()


def mm2s_lane_streams(mem, alignment_sites, window_size, side, layout, aie="window"):
    """Emulate mm2sleft/mm2sright (mem variants): returns a list of 4 lane
    streams, each an (beats, 4) array of 128-bit beats (4 floats).

    side: "left" | "right"; layout: COMBINED | SEPARATE; aie: "window"|"stream".
    For SEPARATE the EV and branch matrices go to side streams; they are
    returned as extra keys in a dict in that case.
    """
    mem = np.asarray(mem)
    words = lambda i: mem[16 * i:16 * i + 16]  # noqa: E731 -- one 512-bit word
    has_ev = not (side == "right" and layout == SEPARATE)
    ev = words(0) if has_ev else None
    pbase = 1 if has_ev else 0
    branch = [transpose4(words(pbase + c)) for c in range(4)]
    dbase = pbase + 4
    lanes = [[] for _ in range(4)]
    side_ev, side_br = [], [[] for _ in range(4)]
    ev_rows = None
    if ev is not None:
        if side == "left":
            ev_rows = [ev[0:4], ev[4:8]]          # mm2sleft Comb:34-35
        else:
            ev_rows = [ev[8:12], ev[12:16]]       # mm2sright Comb: bottom half
    if aie == "stream":
        pad = alignment_sites & 1
        hdr = np.zeros(4, dtype=np.float32)
        hdr[0] = np.float32(alignment_sites + pad)
        for c in range(4):
            lanes[c].append(hdr)
            for r in ev_rows:
                lanes[c].append(r)
            for j in range(4):
                lanes[c].append(branch[c][4 * j:4 * j + 4])
        for i in range(alignment_sites):
            w = words(dbase + i)
            for c in range(4):
                lanes[c].append(w[4 * c:4 * c + 4])
        if pad:
            for c in range(4):
                lanes[c].append(np.zeros(4, dtype=mem.dtype))
        return [np.array(x) for x in lanes]
    apw = window_size >> 4
    nfull = alignment_sites // apw
    nwin = nfull + (alignment_sites - nfull * apw > 0)
    for w in range(nwin):
        if layout == COMBINED:
            for c in range(4):
                for r in ev_rows:
                    lanes[c].append(r)
                for j in range(4):
                    lanes[c].append(branch[c][4 * j:4 * j + 4])
        else:
            for j in range(4):
                if ev is not None:
                    side_ev.append(ev[4 * j:4 * j + 4])
                for c in range(4):
                    side_br[c].append(branch[c][4 * j:4 * j + 4])
        for i in range(apw):
            wd = words(dbase + apw * w + i)
            for c in range(4):
                lanes[c].append(wd[4 * c:4 * c + 4])
    out = [np.array(x) for x in lanes]
    if layout == SEPARATE:
        return dict(data=out, ev=np.array(side_ev) if side_ev else None,
                    branch=[np.array(b) for b in side_br])
    return out


def s2mm(lane_out, alignment_sites, window_size):
    """Emulate s2mm (s2mm_memDNAwindowComb.cpp:20-101): 4 lane output streams
    of (beats,4) -> (CLV words for every padded slot, scaler byte per slot)."""
    apw = window_size >> 4
    nfull = alignment_sites // apw
    nwin = nfull + (alignment_sites - nfull * apw > 0)
    slots = nwin * apw
    dt = lane_out[0].dtype
    mem = np.empty((slots, 16), dtype=dt)
    sc = np.zeros(slots, dtype=np.uint8)
    for s in range(slots):
        x3 = np.concatenate([lane_out[c][s] for c in range(4)]).astype(dt)
        keep = np.all(np.abs(x3.astype(np.float64)) < MINLIKELIHOOD)
        if keep and s < alignment_sites:
            x3 = (x3.astype(np.float64) * TWO_TO_32).astype(dt)
            sc[s] = 1
        mem[s] = x3
    return mem.reshape(-1), sc


def aie_lane_compute(data_left, data_right, branch_left, branch_right, ev):
    """AIE lane arithmetic (mmul_branch x2 -> combine -> ev;
    aie/src/128x9DNAwindow8192Comb/kernels/{mmul_branch,combine,ev}.cpp):
    out = ((x . B_L) * (y . B_R)) . EV with B = P^T as streamed.  float64 here
    (used only as a numpy cross-check of the goldens)."""
    a = data_left.astype(np.float64) @ branch_left.astype(np.float64)
    b = data_right.astype(np.float64) @ branch_right.astype(np.float64)
    return (a * b) @ ev.astype(np.float64)


# --------------------------------------------------------------------------
# AIE golden vectors (aie/data), the reference's own known-answer test.
# --------------------------------------------------------------------------
def _read_rows(path):
    rows = []
    for line in Path(path).read_text().splitlines():
        line = line.strip()
        if line:
            rows.append([float(t) for t in line.split()])
    return np.array(rows, dtype=np.float32)


def parse_aie_kat(data_dir="/root/reference/aie/data"):
    """Parse the AIE stimuli + goldens into plf() inputs for one site.

    Returns dict(EV, left, right, x1, x2, golden) (float32), where
    left[c*16+k*4+l] = B_c[l][k] (inputbranchleft_c holds P_c^T, the matrix the
    AIE multiplies by) and golden[c*4+l] = golden_c row."""
    d = Path(data_dir)
    EV = _read_rows(d / "inputEV0.txt").reshape(16)
    left = np.empty(64, np.float32)
    right = np.empty(64, np.float32)
    x1 = np.empty(16, np.float32)
    x2 = np.empty(16, np.float32)
    golden = np.empty(16, np.float32)
    extras = {}
    for c in range(4):
        BL = _read_rows(d / f"inputbranchleft{c}.txt")
        BR = _read_rows(d / f"inputbranchright{c}.txt")
        left[c * 16:(c + 1) * 16] = BL.T.reshape(16)
        right[c * 16:(c + 1) * 16] = BR.T.reshape(16)
        dl = _read_rows(d / f"inputdataleft{c}.txt")
        dr = _read_rows(d / f"inputdataright{c}.txt")
        g = _read_rows(d / f"golden{c}.txt")
        assert (dl == dl[0]).all() and (dr == dr[0]).all() and (g == g[0]).all()
        x1[c * 4:(c + 1) * 4] = dl[0]
        x2[c * 4:(c + 1) * 4] = dr[0]
        golden[c * 4:(c + 1) * 4] = g[0]
        extras[f"golden_rows{c}"] = len(g)
        extras[f"combinedevleft{c}"] = _read_rows(d / f"inputcombinedevleft{c}.txt")
        extras[f"combinedevright{c}"] = _read_rows(d / f"inputcombinedevright{c}.txt")
        extras[f"stream_combinedevleft{c}"] = _read_rows(d / "stream" / f"inputcombinedevleft{c}.txt")
        extras[f"stream_combinedevright{c}"] = _read_rows(d / "stream" / f"inputcombinedevright{c}.txt")
    return dict(EV=EV, left=left, right=right, x1=x1, x2=x2, golden=golden, **extras)


def compare_rel(a, b, scale=None):
    """max |a-b| / max(|b|) style relative error used by the fp64 tests."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if scale is None:
        scale = np.maximum(np.abs(b), np.finfo(np.float64).tiny)
    return float(np.max(np.abs(a - b) / scale)) if a.size else 0.0
