"""plfx -- Python binding of libplfx.so (include/plfx.h), the MI355X PLF engine.

The binding mirrors the reference's interfaces for the PLF hot path:

* ``plf(x1_start, x2_start, x3_start, EV, n, left, right, wgt)`` -- the
  reference CPU entry point ``plf()`` (/root/reference/app/src/plf.h:1-5):
  same argument order and meaning; the ``int& scalerIncrement`` out-argument
  becomes the return value.  Runs on the GPU through ``plfx_plf_f32/f64``.
* ``plf_dev(...)`` -- the same update on device-resident torch tensors,
  asynchronous on a HIP stream (``plfx_plf_dev_f32/f64``); optional per-site
  scaler bytes (the s2mm char output, hls/src/s2mm_memDNAwindowComb.cpp:97) and
  weighted scaler sum (host_mem.cpp:384-388).
* ``instance_run(...)`` -- the accelerator instance-buffer contract
  (host_mem.cpp:123-157): packed [EV|P_L|CLV_L] / [EV|P_R|CLV_R] or [P_R|CLV_R].
* ``Testbench`` / ``pack_instance`` -- testbench_info sizing
  (app/src/include.h:150-266) and packing (host_mem.cpp:221-243).

There is no CPU fallback: if libplfx.so or a gfx950 device is missing every
call raises ``PlfxError``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libplfx.so"

OK = 0
ERR_INVALID, ERR_HIP, ERR_NOMEM, ERR_NODEV, ERR_UNSUPPORTED = -1, -2, -3, -4, -5
LAYOUT_COMBINED, LAYOUT_SEPARATE = 0, 1
AIE_STREAM, AIE_WINDOW = 0, 1
F32, F64 = 0, 1

# symbols declared by include/plfx.h (checked by tests/test_abi.py)
EXPORTS = (
    "plfx_ctx_create", "plfx_ctx_create_ex", "plfx_ctx_destroy", "plfx_last_error", "plfx_get_version",
    "plfx_ctx_stream", "plfx_ctx_device", "plfx_ctx_synchronize", "plfx_ctx_release_stream",
    "plfx_ctx_set_streams", "plfx_ctx_streams",
    "plfx_plf_f32", "plfx_plf_f64", "plfx_plf_dev_f32", "plfx_plf_dev_f64",
    "plfx_instance_run", "plfx_instance_run_host", "plfx_scaler_sum",
    "plfx_tb_alignments_per_instance", "plfx_tb_alignments_padding",
    "plfx_tb_instance_site_offset", "plfx_tb_elements_per_instance",
    "plfx_tb_instance_elements_left", "plfx_tb_instance_elements_right",
    "plfx_tb_instance_elements_out",
    "plfx_tb_instance_active_elements_left", "plfx_tb_instance_active_elements_right",
    "plfx_tb_num_windows_per_instance", "plfx_pack_instance",
    "plfx_plf_batch_dev", "plfx_traverse", "plfx_root_lnl", "plfx_plf_dev_gen",
    "plfx_plf_tips_dev", "plfx_plf_tips_dev_gen", "plfx_traverse_tips",
    "plfx_model_eigen", "plfx_gamma_rates", "plfx_model_ev", "plfx_model_root_weights",
    "plfx_pmatrix", "plfx_model_tip_vectors",
    "plfx_shard", "plfx_gen_hostmem", "plfx_swemu_instance_run", "plfx_traverse_schedule",
)
MAX_STREAMS = 64   # PLFX_MAX_STREAMS
WS_POOL = 8        # PLFX_WS_POOL
STREAMS_MAX = 8    # PLFX_STREAMS_MAX
STREAM_PER_THREAD = 2  # hipStreamPerThread
SCHED_KEYS = ("deep6", "deep5", "deep4", "septets", "triples", "unfused", "launches")
PMAT_STATE, PMAT_EIGEN = 0, 1
EXACT, FMA = 0, 1
VALU = 2  # with FMA: protein f64 on the VALU, P matrices tiled in LDS (not the matrix cores)
PROT_CODES = 24  # protein tip codes: rows of the tip-vector table (plfx.h section 8)
CTX_LAZY_TABLES = 1  # PLFX_CTX_LAZY_TABLES


class PlfxError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"plfx error {code}: {msg}")
        self.code = code


class Node(C.Structure):
    """plfx_node: one inner-node update (all device pointers)."""
    _fields_ = [("x1", C.c_void_p), ("x2", C.c_void_p), ("x3", C.c_void_p),
                ("left", C.c_void_p), ("right", C.c_void_p), ("scaler", C.c_void_p),
                ("scaler_sum", C.c_void_p)]


class TravOp(C.Structure):
    _fields_ = [("parent", C.c_int32), ("child1", C.c_int32), ("child2", C.c_int32),
                ("pmat", C.c_int32)]


class _TB(C.Structure):
    _fields_ = [("alignment_sites", C.c_uint64), ("parallel_instances", C.c_uint32),
                ("window_size", C.c_uint32), ("layout", C.c_int32), ("aie_type", C.c_int32)]


_lib = None


def load():
    """Load libplfx.so.  torch is imported first (when present) so that the
    library binds to the same HIP runtime instance as torch's allocations."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  -- share torch's libamdhip64
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise PlfxError(ERR_UNSUPPORTED, f"{LIB_PATH} not built (run __graft_entry__.build())")
    L = C.CDLL(str(LIB_PATH))
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int
    L.plfx_ctx_create.argtypes = [i32, C.POINTER(vp)]
    L.plfx_ctx_create_ex.argtypes = [i32, C.c_uint, C.POINTER(vp)]
    L.plfx_ctx_destroy.argtypes = [vp]
    L.plfx_last_error.argtypes = [vp]
    L.plfx_last_error.restype = C.c_char_p
    L.plfx_ctx_stream.argtypes = [vp]
    L.plfx_ctx_stream.restype = vp
    L.plfx_ctx_device.argtypes = [vp]
    L.plfx_ctx_synchronize.argtypes = [vp]
    L.plfx_ctx_release_stream.argtypes = [vp, vp]
    L.plfx_ctx_set_streams.argtypes = [vp, i32]
    L.plfx_ctx_streams.argtypes = [vp]
    for s in ("f32", "f64"):
        getattr(L, f"plfx_plf_{s}").argtypes = [vp, vp, vp, vp, vp, i32, vp, vp, vp, C.POINTER(i32)]
        getattr(L, f"plfx_plf_dev_{s}").argtypes = [vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
    L.plfx_instance_run.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.c_uint32, i32, i32, vp]
    L.plfx_instance_run_host.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.c_uint32, i32, i32]
    L.plfx_scaler_sum.argtypes = [vp, vp, vp, i64, vp, vp]
    tbp = C.POINTER(_TB)
    for name in ("alignments_per_instance", "instance_site_offset",
                 "instance_active_elements_left", "instance_active_elements_right"):
        f = getattr(L, f"plfx_tb_{name}")
        f.argtypes = [tbp, i32]
        f.restype = C.c_uint64
    for name in ("alignments_padding", "elements_per_instance", "instance_elements_left",
                 "instance_elements_right", "instance_elements_out", "num_windows_per_instance"):
        f = getattr(L, f"plfx_tb_{name}")
        f.argtypes = [tbp]
        f.restype = C.c_uint64
    L.plfx_pack_instance.argtypes = [tbp, i32, i32, vp, vp, vp, vp, vp, vp, vp]
    L.plfx_plf_dev_gen.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
    L.plfx_plf_batch_dev.argtypes = [vp, i32, i32, C.POINTER(Node), i32, vp, i64, vp, vp]
    L.plfx_traverse.argtypes = [vp, i32, i32, C.POINTER(TravOp), i32, C.POINTER(vp), i32, vp, i32,
                                vp, i64, vp, C.POINTER(vp), vp, vp]
    L.plfx_root_lnl.argtypes = [vp, i32, i32, vp, i64, vp, vp, vp, vp, i32, vp, vp, vp]
    dp = C.POINTER(C.c_double)
    L.plfx_model_eigen.argtypes = [i32, dp, dp, dp]
    L.plfx_gamma_rates.argtypes = [C.c_double, i32, i32, dp]
    L.plfx_model_ev.argtypes = [i32, i32, dp, dp]
    L.plfx_model_root_weights.argtypes = [i32, i32, dp, dp, dp]
    L.plfx_pmatrix.argtypes = [vp, i32, i32, i32, vp, vp, i32, vp, i64, vp, vp]
    L.plfx_model_tip_vectors.argtypes = [i32, i32, dp, dp]
    L.plfx_plf_tips_dev.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp,
                                    vp]
    L.plfx_plf_tips_dev_gen.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp,
                                        vp, vp, vp, vp]
    L.plfx_traverse_tips.argtypes = [vp, i32, i32, i32, C.POINTER(TravOp), i32, C.POINTER(vp),
                                     C.POINTER(vp), i32, vp, i32, vp, i64, vp, C.POINTER(vp), vp, vp,
                                     vp]
    u64p = C.POINTER(C.c_uint64)
    L.plfx_shard.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, u64p, u64p]
    L.plfx_gen_hostmem.argtypes = [i32, C.c_uint32, C.c_uint64, vp, vp, vp, vp, vp, vp]
    L.plfx_swemu_instance_run.argtypes = [vp, vp, vp, vp, C.c_uint32, C.c_uint32, i32, i32, i32]
    L.plfx_traverse_schedule.argtypes = [vp, C.POINTER(i32), i32]
    _lib = L
    return L


class Context:
    """A libplfx context bound to one HIP device (replaces acap_info,
    app/src/include.h:28-147).  lazy_tables=True (PLFX_CTX_LAZY_TABLES, for
    DNA-only users): the protein tip/tip tables are allocated on a stream's
    first tip/tip call instead of with the context (~95 MB)."""

    def __init__(self, device: int = 0, lazy_tables: bool = False):
        self._L = load()
        h = C.c_void_p()
        rc = self._L.plfx_ctx_create_ex(int(device), CTX_LAZY_TABLES if lazy_tables else 0, C.byref(h))
        if rc != OK:
            raise PlfxError(rc, f"plfx_ctx_create(device={device}) failed "
                                "(no gfx950 device visible?)")
        self.h = h
        self.device = device
        self._used = {}  # torch streams this context ran on: released at close()

    def _sh(self, stream):
        """The hipStream_t of `stream` (None: torch's current stream on the
        context's device), remembering torch streams so that close() can
        release their workspaces (plfx_ctx_release_stream) and destroy stays
        off the device-wide wait.  Raw integer handles are not remembered (the
        stream may be destroyed before the context): release those yourself."""
        if stream is None:
            import torch

            stream = torch.cuda.current_stream(self.device)
        if not isinstance(stream, int):
            self._used[stream.cuda_stream] = stream
        return _stream_handle(stream, self.device)

    def close(self):
        if getattr(self, "h", None):
            for st in list(getattr(self, "_used", {}).values()):
                try:  # refused (and left to destroy) while the stream is being captured
                    self._L.plfx_ctx_release_stream(self.h, C.c_void_p(st.cuda_stream))
                except Exception:
                    pass
            self._used = {}
            self._L.plfx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def stream(self):
        return self._L.plfx_ctx_stream(self.h)

    def synchronize(self):
        self._check(self._L.plfx_ctx_synchronize(self.h))

    @property
    def streams(self):
        """One-node calls kept in flight (plfx_ctx_streams)."""
        return self._L.plfx_ctx_streams(self.h)

    def set_streams(self, streams):
        """Tell the context that `streams` one-node calls run at once, each on
        its own stream (plfx_ctx_set_streams: the dense DNA node and f64
        protein FMA kernels then launch the resident blocks / streams)."""
        self._check(self._L.plfx_ctx_set_streams(self.h, int(streams)))

    def release_stream(self, stream):
        """Wait for `stream` and return its scaler-sum workspace to the pool
        (plfx_ctx_release_stream)."""
        h = _stream_handle(stream, self.device)
        self._check(self._L.plfx_ctx_release_stream(self.h, h))
        self._used.pop(h.value, None)

    def _check(self, rc):
        if rc != OK:
            raise PlfxError(rc, self._L.plfx_last_error(self.h).decode(errors="replace"))

    # -- (1) plf() drop-in on host arrays ----------------------------------
    def plf(self, x1_start, x2_start, x3_start, EV, n, left, right, wgt=None):
        """plf(x1, x2, x3, EV, n, left, right, wgt) -> scalerIncrement.

        numpy float32 or float64 arrays, x3_start written in place."""
        dt = np.asarray(x1_start).dtype
        if dt not in (np.float32, np.float64):
            raise PlfxError(ERR_INVALID, f"unsupported dtype {dt}")
        arrs = [x1_start, x2_start, x3_start, EV, left, right]
        for a in arrs:
            if not (isinstance(a, np.ndarray) and a.dtype == dt and a.flags.c_contiguous):
                raise PlfxError(ERR_INVALID, "arrays must be C-contiguous numpy arrays of one dtype")
        n = int(n)
        if x1_start.size < 16 * n or x2_start.size < 16 * n or x3_start.size < 16 * n:
            raise PlfxError(ERR_INVALID, "CLV arrays shorter than 16*n")
        if EV.size < 16 or left.size < 64 or right.size < 64:
            raise PlfxError(ERR_INVALID, "EV needs 16, left/right 64 values")
        w = None
        if wgt is not None:
            w = np.ascontiguousarray(wgt, dtype=np.int32)
            if w.size < n:
                raise PlfxError(ERR_INVALID, "wgt shorter than n")
        inc = C.c_int(0)
        fn = self._L.plfx_plf_f32 if dt == np.float32 else self._L.plfx_plf_f64
        p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
        self._check(fn(self.h, p(x1_start), p(x2_start), p(x3_start), p(EV), n, p(left), p(right),
                       p(w), C.byref(inc)))
        return inc.value

    # -- (2) device-resident hot path ---------------------------------------
    def plf_dev(self, x1, x2, x3, EV, left, right, wgt=None, scaler=None, scaler_sum=None,
                n=None, stream=None):
        """Fused PLF on torch device tensors (float32/float64, contiguous).

        Asynchronous on `stream` (a torch.cuda.Stream, a raw hipStream_t int,
        or None = torch's current stream)."""
        import torch

        dt = x1.dtype
        if dt not in (torch.float32, torch.float64):
            raise PlfxError(ERR_INVALID, f"unsupported dtype {dt}")
        for t in (x1, x2, x3, EV, left, right):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise PlfxError(ERR_INVALID, "tensors must be contiguous device tensors of one dtype")
        if n is None:
            n = x1.numel() // 16
        n = int(n)
        if min(x1.numel(), x2.numel(), x3.numel()) < 16 * n:
            raise PlfxError(ERR_INVALID, "CLV tensors shorter than 16*n")
        if EV.numel() < 16 or left.numel() < 64 or right.numel() < 64:
            raise PlfxError(ERR_INVALID, "EV needs 16, left/right 64 values")
        _check_aux(n, wgt, scaler, scaler_sum)
        fn = self._L.plfx_plf_dev_f32 if dt == torch.float32 else self._L.plfx_plf_dev_f64
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(fn(self.h, p(x1), p(x2), p(x3), p(EV), n, p(left), p(right), p(wgt),
                       p(scaler), p(scaler_sum), self._sh(stream)))

    def bind_plf_dev(self, x1, x2, x3, EV, left, right, wgt=None, scaler=None, scaler_sum=None,
                     n=None):
        """Validate once and return a launcher ``run(stream=None)`` that issues
        the same fused PLF call with no per-call Python checks (for launch-rate
        bound loops: a 1M-site f64 call is ~67 us of GPU time).  The launcher
        holds references to the tensors, so their memory stays allocated while
        it lives (a graph captured through it, too, needs it alive); the
        tensors must keep their shape and device."""
        import torch

        self.plf_dev(x1, x2, x3, EV, left, right, wgt, scaler, scaler_sum, n=n,
                     stream=torch.cuda.current_stream(x1.device).cuda_stream)  # validates
        n = x1.numel() // 16 if n is None else int(n)
        fn = self._L.plfx_plf_dev_f32 if x1.dtype == torch.float32 else self._L.plfx_plf_dev_f64
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        args = (self.h, p(x1), p(x2), p(x3), p(EV), C.c_int64(n), p(left), p(right), p(wgt),
                p(scaler), p(scaler_sum))
        check = self._check
        held = (x1, x2, x3, EV, left, right, wgt, scaler, scaler_sum)  # raw pointers in args

        def run(stream=None):
            if self.h is None:  # args carry the handle: a closed context's would dangle
                raise PlfxError(ERR_INVALID, "launcher used after its context was closed")
            check(fn(*args, self._sh(stream)))

        run.tensors = held
        return run

    # -- (3) instance-buffer contract --------------------------------------
    def instance_run(self, in_left, in_right, out_clv, out_scaler, alignment_sites, window_size,
                     layout, stream=None):
        import torch

        dt = in_left.dtype
        if dt not in (torch.float32, torch.float64) or in_right.dtype != dt or out_clv.dtype != dt:
            raise PlfxError(ERR_INVALID, "instance buffers must share a float dtype")
        hdr_r = 80 if layout == LAYOUT_COMBINED else 64
        n = int(alignment_sites)
        if in_left.numel() < 80 + 16 * n or in_right.numel() < hdr_r + 16 * n or \
                out_clv.numel() < 16 * n:
            raise PlfxError(ERR_INVALID, "instance buffers too small for alignment_sites")
        if out_scaler is not None and (out_scaler.dtype != torch.uint8 or out_scaler.numel() < n):
            raise PlfxError(ERR_INVALID, "out_scaler must be uint8 with >= alignment_sites bytes")
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self._L.plfx_instance_run(self.h, p(in_left), p(in_right), p(out_clv),
                                              p(out_scaler), n, int(window_size), int(layout),
                                              F32 if dt == torch.float32 else F64,
                                              self._sh(stream)))

    def instance_run_host(self, in_left, in_right, out_clv, out_scaler, alignment_sites,
                          window_size, layout):
        """instance_run on numpy host buffers, synchronous (bo.write -> run ->
        bo.read, host_mem.cpp:293-318)."""
        import numpy as np

        dt = in_left.dtype
        if dt not in (np.float32, np.float64) or in_right.dtype != dt or out_clv.dtype != dt:
            raise PlfxError(ERR_INVALID, "instance buffers must share a float dtype")
        hdr_r = 80 if layout == LAYOUT_COMBINED else 64
        n = int(alignment_sites)
        if in_left.size < 80 + 16 * n or in_right.size < hdr_r + 16 * n or out_clv.size < 16 * n:
            raise PlfxError(ERR_INVALID, "instance buffers too small for alignment_sites")
        if out_scaler is not None and (out_scaler.dtype != np.uint8 or out_scaler.size < n):
            raise PlfxError(ERR_INVALID, "out_scaler must be uint8 with >= alignment_sites bytes")
        for a in (in_left, in_right, out_clv, out_scaler):
            if a is not None and not a.flags.c_contiguous:
                raise PlfxError(ERR_INVALID, "instance buffers must be C-contiguous")
        p = lambda a: None if a is None else C.c_void_p(a.ctypes.data)  # noqa: E731
        self._check(self._L.plfx_instance_run_host(self.h, p(in_left), p(in_right), p(out_clv),
                                                   p(out_scaler), n, int(window_size), int(layout),
                                                   F32 if dt == np.float32 else F64))

    def plf_dev_gen(self, x1, x2, x3, EV, left, right, states, wgt=None, scaler=None,
                    scaler_sum=None, n=None, fma=False, stream=None, valu=False):
        """Any built state count (4 DNA, 20 protein), 4 Gamma categories, on
        torch device tensors: x[site][cat][state], P [cat][k][l], EV [k][l].
        fma: PLFX_FMA; valu (with fma, protein f64): the same fused chains on
        the VALU with LDS-tiled matrices instead of the matrix cores
        (PLFX_VALU; bit-identical)."""
        import torch

        V = 4 * states
        dt = x1.dtype
        if dt not in (torch.float32, torch.float64):
            raise PlfxError(ERR_INVALID, f"unsupported dtype {dt}")
        if n is None:
            n = x1.numel() // V
        n = int(n)
        for t in (x1, x2, x3, EV, left, right):
            if t.dtype != dt or not t.is_cuda or not t.is_contiguous():
                raise PlfxError(ERR_INVALID, "tensors must be contiguous device tensors of one dtype")
        if min(x1.numel(), x2.numel(), x3.numel()) < V * n:
            raise PlfxError(ERR_INVALID, "CLV tensors shorter than 4*states*n")
        if EV.numel() < states * states or min(left.numel(), right.numel()) < 4 * states * states:
            raise PlfxError(ERR_INVALID, "EV needs S*S, left/right 4*S*S values")
        _check_aux(n, wgt, scaler, scaler_sum)
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self._L.plfx_plf_dev_gen(self.h, F32 if dt == torch.float32 else F64, int(states),
                                             (FMA if fma else EXACT) | (VALU if valu else 0),
                                             p(x1), p(x2), p(x3), p(EV), n,
                                             p(left), p(right), p(wgt), p(scaler), p(scaler_sum),
                                             self._sh(stream)))

    # -- (6) batched nodes / traversal ---------------------------------------
    def plf_batch_dev(self, nodes, EV, n, wgt=None, stream=None, states=4):
        """nodes: sequence of dicts with torch tensors x1, x2, x3, left, right and
        optional scaler (uint8[n]), scaler_sum (int64[1]); all one float dtype,
        all sharing EV, n (sites) and wgt."""
        import torch

        dt = EV.dtype
        V, M = 4 * states, 4 * states * states
        arr = (Node * len(nodes))()
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        for i, nd in enumerate(nodes):
            for k in ("x1", "x2", "x3"):
                t = nd[k]
                if t.dtype != dt or t.numel() < V * n or not t.is_contiguous() or not t.is_cuda:
                    raise PlfxError(ERR_INVALID, f"node {i}: {k} must be a contiguous {dt} device "
                                                 f"tensor >= {V}*n")
            for k in ("left", "right"):
                if nd[k].dtype != dt or nd[k].numel() < M or not nd[k].is_cuda or not nd[k].is_contiguous():
                    raise PlfxError(ERR_INVALID, f"node {i}: {k} needs {M} contiguous device values")
            try:
                _check_aux(n, None, nd.get("scaler"), nd.get("scaler_sum"))
            except PlfxError as e:
                raise PlfxError(ERR_INVALID, f"node {i}: {e}") from None
            arr[i] = Node(ptr(nd["x1"]), ptr(nd["x2"]), ptr(nd["x3"]), ptr(nd["left"]),
                          ptr(nd["right"]), ptr(nd.get("scaler")), ptr(nd.get("scaler_sum")))
        _check_aux(n, wgt, None, None)
        if not EV.is_cuda or not EV.is_contiguous() or EV.numel() < states * states:
            raise PlfxError(ERR_INVALID, f"EV must be a contiguous device tensor of {states * states} values")
        self._check(self._L.plfx_plf_batch_dev(self.h, F32 if dt == torch.float32 else F64, states, arr,
                                               len(nodes), C.c_void_p(EV.data_ptr()), int(n),
                                               C.c_void_p(ptr(wgt)), self._sh(stream)))

    def bind_plf_batch_dev(self, nodes, EV, n, wgt=None, states=4):
        """Validate once (as plf_batch_dev) and return a launcher
        ``run(stream=None)`` issuing the same batched call with a prebuilt
        node array (graph capture / launch-rate bound loops).  The launcher
        holds references to every node's tensors, EV and wgt, so their memory
        stays allocated while it lives."""
        import torch

        if not nodes:
            return lambda stream=None: None
        self.plf_batch_dev(nodes, EV, n, wgt, stream=torch.cuda.current_stream(self.device).cuda_stream,
                           states=states)  # validates
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        arr = (Node * len(nodes))(*[Node(ptr(nd["x1"]), ptr(nd["x2"]), ptr(nd["x3"]), ptr(nd["left"]),
                                         ptr(nd["right"]), ptr(nd.get("scaler")),
                                         ptr(nd.get("scaler_sum"))) for nd in nodes])
        fn, h, check = self._L.plfx_plf_batch_dev, self.h, self._check
        args = (F32 if EV.dtype == torch.float32 else F64, states, arr, len(nodes),
                C.c_void_p(EV.data_ptr()), int(n), C.c_void_p(ptr(wgt)))

        ctx = self

        def run(stream=None):
            if ctx.h is None:  # h would dangle
                raise PlfxError(ERR_INVALID, "launcher used after its context was closed")
            check(fn(h, *args, ctx._sh(stream)))

        run.tensors = ([dict(nd) for nd in nodes], EV, wgt)  # raw pointers in arr / args
        return run

    def traverse(self, ops, clv, pmats, EV, n, wgt=None, scalers=None, scaler_sums=None,
                 stream=None, tips=None, tipvec=None, states=4, fma=False):
        """Run a post-order traversal descriptor.  ops: (nops, 4) int array of
        [parent, child1, child2, pmat]; clv: list of torch CLV tensors (slots;
        None where the slot is a tip); pmats: tensor of 2*npmat matrices (64
        values each for DNA); tips: optional list (per slot) of uint8 code
        tensors or None (plfx.h section 8: DNA state bits, protein code
        indices); tipvec: optional device table of tip vectors (16 x 4 DNA,
        PROT_CODES x 20 protein; dtype of the CLVs); states 4 or 20, fma:
        PLFX_FMA for protein nodes."""
        import torch

        ops = np.ascontiguousarray(ops, dtype=np.int32).reshape(-1, 4)
        nops = ops.shape[0]
        dt = EV.dtype
        nslots = len(clv)
        if tips is not None and len(tips) != nslots:
            raise PlfxError(ERR_INVALID, "tips must have one entry per slot")
        V, M = 4 * states, 4 * states * states
        for s_, t in enumerate(clv):
            tip = None if tips is None else tips[s_]
            if tip is not None:
                if tip.dtype != torch.uint8 or tip.numel() < n or not tip.is_contiguous() or not tip.is_cuda:
                    raise PlfxError(ERR_INVALID, f"tip slot {s_}: contiguous uint8 >= n required")
                continue
            if t is None or t.dtype != dt or t.numel() < V * n or not t.is_contiguous() or not t.is_cuda:
                raise PlfxError(ERR_INVALID, f"every CLV slot must be a contiguous device tensor, "
                                             f"same dtype, >= {V}*n")
        if pmats.dtype != dt or pmats.numel() % (2 * M):
            raise PlfxError(ERR_INVALID, f"pmats must hold whole (left, right) pairs of {M} values")
        if scaler_sums is not None and (scaler_sums.dtype != torch.int64 or scaler_sums.numel() < nops
                                        or not scaler_sums.is_cuda):
            raise PlfxError(ERR_INVALID, "scaler_sums must be an int64 device tensor with >= nops entries")
        if scalers is not None:
            if len(scalers) > nops:
                raise PlfxError(ERR_INVALID, "more scaler tensors than ops")
            scalers = list(scalers) + [None] * (nops - len(scalers))
            for j, t in enumerate(scalers):
                if t is not None and (t.dtype != torch.uint8 or not t.is_cuda or not t.is_contiguous()
                                      or t.numel() < n):
                    raise PlfxError(ERR_INVALID, f"scaler of op {j} must be a contiguous uint8 "
                                                 f"device tensor of >= n elements")
        _check_aux(n, wgt, None, None)
        for t in (pmats, EV):
            if not t.is_cuda or not t.is_contiguous():
                raise PlfxError(ERR_INVALID, "pmats and EV must be contiguous device tensors")
        if EV.numel() < states * states:
            raise PlfxError(ERR_INVALID, f"EV needs {states * states} values")
        top = (TravOp * nops)(*[TravOp(*map(int, r)) for r in ops])
        slots = (C.c_void_p * nslots)(*[None if t is None else t.data_ptr() for t in clv])
        tp = None
        if tips is not None:
            tp = (C.c_void_p * nslots)(*[None if t is None else t.data_ptr() for t in tips])
        sc = None
        if scalers is not None:
            sc = (C.c_void_p * nops)(*[None if t is None else t.data_ptr() for t in scalers])
        self._check(self._L.plfx_traverse_tips(
            self.h, F32 if dt == torch.float32 else F64, states, FMA if fma else EXACT, top, nops,
            slots, tp, nslots, C.c_void_p(pmats.data_ptr()), pmats.numel() // (2 * M),
            C.c_void_p(EV.data_ptr()), int(n),
            C.c_void_p(None if wgt is None else wgt.data_ptr()), sc,
            C.c_void_p(None if scaler_sums is None else scaler_sums.data_ptr()),
            self._tipvec(tipvec, dt, states), self._sh(stream)))

    @staticmethod
    def _tipvec(tipvec, dt, states=4):
        if tipvec is None:
            return C.c_void_p(None)
        rows, width = (16, 4) if states == 4 else (PROT_CODES, 20)
        if tipvec.dtype != dt or tipvec.numel() < rows * width or not tipvec.is_contiguous():
            raise PlfxError(ERR_INVALID, f"tipvec must be a contiguous device table of "
                                         f"{rows} x {width} values")
        return C.c_void_p(tipvec.data_ptr())

    def plf_tips_dev(self, x3, EV, n, left, right, x1=None, x2=None, tip1=None, tip2=None,
                     wgt=None, scaler=None, scaler_sum=None, tipvec=None, stream=None, states=4,
                     fma=False):
        """One inner node with tip children (plfx.h section 8): for each child
        pass exactly one of the dense CLV (x1/x2) or the uint8 codes
        (tip1/tip2).  states 4 (DNA state bits) or 20 (protein code indices,
        PROT_CODES rows); fma: PLFX_FMA (protein)."""
        import torch

        dt = EV.dtype
        V = 4 * states
        for k, t in (("x3", x3), ("x1", x1), ("x2", x2)):
            if t is not None and (t.dtype != dt or t.numel() < V * n or not t.is_contiguous()
                                  or not t.is_cuda):
                raise PlfxError(ERR_INVALID, f"{k} must be a contiguous {dt} device tensor >= {V}*n")
        for k, t in (("tip1", tip1), ("tip2", tip2)):
            if t is not None and (t.dtype != torch.uint8 or t.numel() < n or not t.is_contiguous()
                                  or not t.is_cuda):
                raise PlfxError(ERR_INVALID, f"{k} must be a contiguous uint8 device tensor >= n")
        for k, t in (("EV", EV), ("left", left), ("right", right)):
            if t.dtype != dt or not t.is_cuda or t.numel() < (states * states if k == "EV"
                                                               else 4 * states * states):
                raise PlfxError(ERR_INVALID, f"{k} must be a {dt} device tensor of the model's size")
        _check_aux(n, wgt, scaler, scaler_sum)
        p = lambda t: C.c_void_p(None if t is None else t.data_ptr())  # noqa: E731
        self._check(self._L.plfx_plf_tips_dev_gen(
            self.h, F32 if dt == torch.float32 else F64, states, FMA if fma else EXACT, p(tip1),
            p(x1), p(tip2), p(x2), p(x3), p(EV), int(n), p(left), p(right), p(wgt), p(scaler),
            p(scaler_sum), self._tipvec(tipvec, dt, states), self._sh(stream)))

    def last_schedule(self):
        """The schedule the last traverse() on this context chose
        (plfx_traverse_schedule): dict over SCHED_KEYS."""
        c = (C.c_int * len(SCHED_KEYS))()
        m = self._L.plfx_traverse_schedule(self.h, c, len(SCHED_KEYS))
        return {k: int(c[i]) for i, k in enumerate(SCHED_KEYS[:m])}

    # -- (9) P matrices from branch lengths --------------------------------
    def pmatrix(self, eigen, rates, blen, out, states=4, convention=PMAT_STATE, stream=None):
        """out[b][c][k][l] from a device eigensystem (float64, S+2S^2), device
        category rates (float64) and branch lengths (float64); plfx.h (9)."""
        import torch

        S = states
        for k, t in (("eigen", eigen), ("rates", rates), ("blen", blen)):
            if t.dtype != torch.float64 or not t.is_contiguous() or not t.is_cuda:
                raise PlfxError(ERR_INVALID, f"{k} must be a contiguous float64 device tensor")
        if eigen.numel() < S + 2 * S * S:
            raise PlfxError(ERR_INVALID, "eigen too small")
        ncat, nb = rates.numel(), blen.numel()
        if (out.dtype not in (torch.float32, torch.float64) or out.numel() < nb * ncat * S * S
                or not out.is_cuda or not out.is_contiguous()):
            raise PlfxError(ERR_INVALID, "out must be a contiguous device tensor of nbranch*ncat*S*S "
                                         "float values")
        self._check(self._L.plfx_pmatrix(
            self.h, F32 if out.dtype == torch.float32 else F64, S, convention,
            C.c_void_p(eigen.data_ptr()), C.c_void_p(rates.data_ptr()), ncat,
            C.c_void_p(blen.data_ptr()), nb, C.c_void_p(out.data_ptr()), self._sh(stream)))

    # -- (7) root log-likelihood --------------------------------------------
    def root_lnl(self, x, n, out, catw=None, freq=None, wgt=None, scaler_sums=None,
                 site_lnl=None, states=4, stream=None):
        """Root lnL into `out` (float64 device tensor, 1 element); see plfx.h (7)."""
        import torch

        if out.dtype != torch.float64 or out.numel() < 1 or not out.is_cuda:
            raise PlfxError(ERR_INVALID, "out must be a float64 device tensor")
        if (x.dtype not in (torch.float32, torch.float64) or x.numel() < 4 * states * n
                or not x.is_cuda or not x.is_contiguous()):
            raise PlfxError(ERR_INVALID, "x must be a contiguous float device tensor of >= 4*S*n values")
        for t, k in ((catw, 4), (freq, states), (site_lnl, n)):
            if t is not None and (t.dtype != torch.float64 or t.numel() < k or not t.is_cuda
                                  or not t.is_contiguous()):
                raise PlfxError(ERR_INVALID, "catw/freq/site_lnl must be contiguous float64 device "
                                             "tensors (4 / S / n values)")
        _check_aux(n, wgt, None, None)
        if scaler_sums is not None and (scaler_sums.dtype != torch.int64 or not scaler_sums.is_cuda
                                        or not scaler_sums.is_contiguous()):
            raise PlfxError(ERR_INVALID, "scaler_sums must be a contiguous int64 device tensor")
        p = lambda t: C.c_void_p(None if t is None else t.data_ptr())  # noqa: E731
        nsums = 0 if scaler_sums is None else scaler_sums.numel()
        self._check(self._L.plfx_root_lnl(self.h, F32 if x.dtype == torch.float32 else F64, states,
                                          p(x), int(n), p(catw), p(freq), p(wgt), p(scaler_sums),
                                          nsums, p(out), p(site_lnl), self._sh(stream)))

    # -- (4) scaler reduction ----------------------------------------------
    def scaler_sum(self, scaler, wgt, out_sum, n=None, stream=None):
        import torch

        if n is None:
            n = scaler.numel()
        if scaler.dtype != torch.uint8 or out_sum.dtype != torch.int64:
            raise PlfxError(ERR_INVALID, "scaler uint8, out_sum int64")
        _check_aux(n, wgt, scaler, out_sum)
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self._L.plfx_scaler_sum(self.h, p(scaler), p(wgt), int(n), p(out_sum),
                                            self._sh(stream)))


def _stream_handle(stream, device=None):
    """None = torch's current stream ON THE CONTEXT'S DEVICE (not the current
    device's), a torch.cuda.Stream, or a raw hipStream_t int."""
    if stream is None:
        import torch

        return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def _check_aux(n, wgt, scaler, scaler_sum):
    """Shapes/dtypes/devices of the optional per-site weight, scaler bytes and
    scaler-sum outputs (the C ABI cannot see tensor sizes)."""
    import torch

    if wgt is not None and (wgt.dtype != torch.int32 or wgt.numel() < n or not wgt.is_cuda
                            or not wgt.is_contiguous()):
        raise PlfxError(ERR_INVALID, "wgt must be a contiguous int32 device tensor of >= n elements")
    if scaler is not None and (scaler.dtype != torch.uint8 or scaler.numel() < n or not scaler.is_cuda
                               or not scaler.is_contiguous()):
        raise PlfxError(ERR_INVALID, "scaler must be a contiguous uint8 device tensor of >= n elements")
    if scaler_sum is not None and (scaler_sum.dtype != torch.int64 or scaler_sum.numel() < 1
                                   or not scaler_sum.is_cuda):
        raise PlfxError(ERR_INVALID, "scaler_sum must be an int64 device tensor")


def shard(total, parts, k):
    """The reference's partition (include.h:181-189; host_mem.cpp:229): part k
    of `total` items over `parts` -> (offset, count).  Used for inner nodes
    over ranks (BASELINE configs[3]) and sites over instances."""
    off, cnt = C.c_uint64(0), C.c_uint64(0)
    rc = load().plfx_shard(int(total), int(parts), int(k), C.byref(off), C.byref(cnt))
    if rc != OK:
        raise PlfxError(rc, f"plfx_shard({total}, {parts}, {k}): the reference's split underflows")
    return int(off.value), int(cnt.value)


def gen_hostmem(n, dtype=np.float64, seed=20250117, wgt=True):
    """host_mem.cpp:179-209 inputs (std::mt19937 + uniform_real_distribution,
    x1 x 1e-12 on every 4th site, wgt = 1) with a fixed seed, generated by
    libplfx (plfx_gen_hostmem).  Returns dict(EV, left, right, x1, x2, wgt)."""
    dt = np.dtype(dtype)
    out = dict(EV=np.empty(16, dt), left=np.empty(64, dt), right=np.empty(64, dt),
               x1=np.empty(16 * n, dt), x2=np.empty(16 * n, dt),
               wgt=np.empty(n, np.int32) if wgt else None)
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = load().plfx_gen_hostmem(F32 if dt == np.float32 else F64, int(seed), int(n), p(out["EV"]),
                                 p(out["left"]), p(out["right"]), p(out["x1"]), p(out["x2"]),
                                 p(out["wgt"]))
    if rc != OK:
        raise PlfxError(rc, "plfx_gen_hostmem")
    return out


def swemu_instance_run(in_left, in_right, out_clv, out_scaler, alignment_sites, window_size,
                       layout, aie_type=AIE_WINDOW):
    """The sw_emu target (plfx.h section 5b, BASELINE configs[0]): one
    accelerator instance emulated on the CPU as its dataflow -- movers, AIE
    lanes, s2mm -- over the whole padded host instance buffers.  No GPU."""
    dt = in_left.dtype
    if dt not in (np.float32, np.float64) or in_right.dtype != dt or out_clv.dtype != dt:
        raise PlfxError(ERR_INVALID, "instance buffers must share a float dtype")
    for a in (in_left, in_right, out_clv, out_scaler):
        if a is not None and not (isinstance(a, np.ndarray) and a.flags.c_contiguous):
            raise PlfxError(ERR_INVALID, "instance buffers must be C-contiguous numpy arrays")
    n = int(alignment_sites)
    tb = Testbench(n, 1, window_size or 1024, layout, aie_type)
    if in_left.size < tb.instance_elements_left() or in_right.size < tb.instance_elements_right() \
            or out_clv.size < 16 * n or (out_scaler is not None and out_scaler.size < n):
        raise PlfxError(ERR_INVALID, "buffers smaller than the padded instance")
    p = lambda a: None if a is None else C.c_void_p(a.ctypes.data)  # noqa: E731
    rc = load().plfx_swemu_instance_run(p(in_left), p(in_right), p(out_clv), p(out_scaler), n,
                                        int(window_size), int(layout), int(aie_type),
                                        F32 if dt == np.float32 else F64)
    if rc != OK:
        raise PlfxError(rc, "plfx_swemu_instance_run")


_default_ctx = None


def _dbl(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


def _host_check(rc, what):
    if rc != OK:
        raise PlfxError(rc, what)


def model_eigen(exch, freqs):
    """Eigensystem of a time-reversible model (plfx.h (9)).  Returns a float64
    array lambda[S] | V[S*S] | Vinv[S*S] (the device pmatrix input)."""
    L = load()
    f, fp = _dbl(freqs)
    S = f.size
    e, ep = _dbl(exch)
    if e.size != S * (S - 1) // 2:
        raise PlfxError(ERR_INVALID, "exch needs S(S-1)/2 values")
    out, op = _dbl(np.zeros(S + 2 * S * S))
    _host_check(L.plfx_model_eigen(S, ep, fp, op), "model_eigen")
    return out


def gamma_rates(alpha, ncat=4, median=False):
    """Yang (1994) discrete-Gamma category rates (plfx.h (9))."""
    L = load()
    out, op = _dbl(np.zeros(ncat))
    _host_check(L.plfx_gamma_rates(float(alpha), int(ncat), 1 if median else 0, op), "gamma_rates")
    return out


def model_ev(eigen, states, convention=PMAT_STATE):
    L = load()
    e, ep = _dbl(eigen)
    out, op = _dbl(np.zeros(states * states))
    _host_check(L.plfx_model_ev(states, convention, ep, op), "model_ev")
    return out


def model_root_weights(eigen, freqs, convention=PMAT_STATE):
    L = load()
    f, fp = _dbl(freqs)
    e, ep = _dbl(eigen)
    out, op = _dbl(np.zeros(f.size))
    _host_check(L.plfx_model_root_weights(f.size, convention, ep, fp, op), "model_root_weights")
    return out


def model_tip_vectors(eigen=None, convention=PMAT_STATE, states=4):
    """16 x S tip vectors for the tip paths (plfx.h (9))."""
    L = load()
    out, op = _dbl(np.zeros(16 * states))
    if eigen is None:
        ep = C.cast(None, C.POINTER(C.c_double))
    else:
        e, ep = _dbl(eigen)
    _host_check(L.plfx_model_tip_vectors(states, convention, ep, op), "model_tip_vectors")
    return out


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def plf(x1_start, x2_start, x3_start, EV, n, left, right, wgt=None):
    """Module-level drop-in for the reference plf() (app/src/plf.h:1-5) on the
    default context.  Returns scalerIncrement."""
    return default_context().plf(x1_start, x2_start, x3_start, EV, n, left, right, wgt)


class Testbench:
    """testbench_info (app/src/include.h:150-266) via the C ABI (64-bit)."""

    def __init__(self, alignment_sites, parallel_instances=1, window_size=1024,
                 layout=LAYOUT_SEPARATE, aie_type=AIE_WINDOW):
        self._L = load()
        self.t = _TB(int(alignment_sites), int(parallel_instances), int(window_size), int(layout),
                     int(aie_type))

    def __getattr__(self, name):
        f = getattr(self._L, f"plfx_tb_{name}", None)
        if f is None:
            raise AttributeError(name)
        if len(f.argtypes) == 2:
            return lambda k=-1: int(f(C.byref(self.t), int(k)))
        return lambda: int(f(C.byref(self.t)))

    def pack_instance(self, k, EV, left, right, x1, x2):
        dt = np.asarray(x1).dtype
        L = np.empty(self.instance_elements_left(), dt)
        R = np.empty(self.instance_elements_right(), dt)
        keep = [np.ascontiguousarray(a, dt) for a in (EV, left, right, x1, x2)]
        rc = self._L.plfx_pack_instance(C.byref(self.t), int(k), F32 if dt == np.float32 else F64,
                                        *[a.ctypes.data_as(C.c_void_p) for a in keep],
                                        L.ctypes.data_as(C.c_void_p), R.ctypes.data_as(C.c_void_p))
        if rc != OK:
            raise PlfxError(rc, "plfx_pack_instance failed")
        return L, R
