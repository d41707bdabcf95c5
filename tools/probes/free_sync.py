#!/usr/bin/env python3
"""Which HIP calls wait for unrelated device work (plfx_ctx_destroy must not):
a ~1 s spin kernel on one torch stream, then each call timed from the host.
  python3 tools/probes/free_sync.py"""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
t0 = time.perf_counter()
torch.cuda._sleep(50_000_000)
torch.cuda.synchronize()
rate = 50_000_000 / (time.perf_counter() - t0)
other = torch.cuda.Stream()


def busy_then(name, fn):
    with torch.cuda.stream(other):
        torch.cuda._sleep(int(1.0 * rate))
    ev = torch.cuda.Event()
    ev.record(other)
    t = time.perf_counter()
    rc = fn()
    dt = time.perf_counter() - t
    print(f"{name:40s} rc={rc} {dt * 1e3:8.2f} ms  other_still_busy={not ev.query()}", flush=True)
    torch.cuda.synchronize()


s = ctypes.c_void_p()
hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
p = ctypes.c_void_p()
hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 24))
busy_then("hipFree (16 MiB)", lambda: hip.hipFree(p))
hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 24))
busy_then("hipMalloc (16 MiB)", lambda: hip.hipMalloc(ctypes.byref(ctypes.c_void_p()), ctypes.c_size_t(1 << 24)))
q = ctypes.c_void_p()
hip.hipMallocAsync(ctypes.byref(q), ctypes.c_size_t(1 << 24), s)
hip.hipStreamSynchronize(s)
busy_then("hipFreeAsync (16 MiB) on own stream", lambda: hip.hipFreeAsync(q, s))
busy_then("hipStreamSynchronize(own)", lambda: hip.hipStreamSynchronize(s))
busy_then("hipStreamDestroy(own)", lambda: hip.hipStreamDestroy(s))
e = ctypes.c_void_p()
hip.hipEventCreateWithFlags(ctypes.byref(e), 2)
busy_then("hipEventDestroy", lambda: hip.hipEventDestroy(e))
h = ctypes.c_void_p()
hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(1 << 20), 0)
busy_then("hipHostFree", lambda: hip.hipHostFree(h))
hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
busy_then("hipFree (pool block) then nothing", lambda: hip.hipFree(p))
