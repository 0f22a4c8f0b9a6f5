"""Probe (GPU box): cost of page-locking host memory and the D2H / H2D link
rates the drop-in batch path (hbam_decode_span) is built on.

  * hipHostMalloc of 64 MiB .. 1 GiB (torch pin_memory allocations, fresh);
  * malloc + first touch on T threads + hipHostRegister of the same sizes;
  * D2H into page-locked memory alone, H2D alone, both at once on two
    streams (full duplex?), and D2H into pageable memory.
Prints one JSON line."""
import ctypes
import json
import time

import numpy as np
import torch

MiB = 1 << 20
out = {}
torch.cuda.init()
torch.empty(1, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")

for mb in (64, 256, 1024):
    n = mb * MiB
    t = time.perf_counter()
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0) == 0
    dt = time.perf_counter() - t
    hip.hipHostFree(p)
    out[f"hipHostMalloc_{mb}MiB_ms"] = round(dt * 1e3, 2)
    a = np.empty(n, np.uint8)
    t = time.perf_counter()
    a[::4096] = 1  # first touch of every page
    t1 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(n), 0)
    t2 = time.perf_counter()
    out[f"touch_{mb}MiB_ms"] = round((t1 - t) * 1e3, 2)
    out[f"hipHostRegister_{mb}MiB_ms"] = round((t2 - t1) * 1e3, 2) if rc == 0 else f"rc={rc}"
    if rc == 0:
        hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))
    del a

n = 1024 * MiB
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
dev2 = torch.empty(n, dtype=torch.uint8, device="cuda")
h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.ones(n, dtype=torch.uint8, pin_memory=True)
hp = torch.empty(n, dtype=torch.uint8)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def d2h():
    with torch.cuda.stream(s1):
        h1.copy_(dev, non_blocking=True)


def h2d():
    with torch.cuda.stream(s2):
        dev2.copy_(h2, non_blocking=True)


out["d2h_pinned_GBps"] = round(n / timed(d2h) / 1e9, 2)
out["h2d_pinned_GBps"] = round(n / timed(h2d) / 1e9, 2)
both = timed(lambda: (d2h(), h2d()))
out["duplex_GBps_each"] = round(n / both / 1e9, 2)
out["d2h_pageable_GBps"] = round(n / timed(lambda: hp.copy_(dev)) / 1e9, 2)
print(json.dumps(out), flush=True)
