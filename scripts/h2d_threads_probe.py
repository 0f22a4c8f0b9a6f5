"""Pageable host->HBM copy rate of a mapped /dev/shm file: one copy vs several
threads each copying a slice on its own stream, and page-locked bounce
buffers filled by host threads (the candidates for Pipeline::stage)."""
import os, sys, time, threading
import numpy as np
import torch

GB = 4 << 30
path = "/dev/shm/h2d_probe.bin"
with open(path, "wb") as f:
    f.truncate(GB)
m = np.memmap(path, dtype=np.uint8, mode="r+")
m[::4096] = 1  # fault the pages in (the C3 leg prefetches too)
src = torch.from_numpy(np.asarray(m))
dev = torch.empty(GB, dtype=torch.uint8, device="cuda:0")
torch.cuda.synchronize()


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def one():
    dev.copy_(src)


def threads(n):
    def run():
        step = GB // n
        streams = [torch.cuda.Stream() for _ in range(n)]

        def part(i):
            with torch.cuda.stream(streams[i]):
                dev[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step])
                streams[i].synchronize()

        ts = [threading.Thread(target=part, args=(i,)) for i in range(n)]
        [t.start() for t in ts]
        [t.join() for t in ts]
    return run


def bounce(nthreads, chunk=256 << 20):
    bufs = [torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(2)]
    s = torch.cuda.Stream()
    evs = [torch.cuda.Event() for _ in range(2)]

    def fill(dst, lo, n):
        step = (n + nthreads - 1) // nthreads

        def w(i):
            a = i * step
            b = min(n, a + step)
            if a < b:
                dst[a:b].copy_(src[lo + a:lo + b])
        ts = [threading.Thread(target=w, args=(i,)) for i in range(nthreads)]
        [t.start() for t in ts]
        [t.join() for t in ts]

    def run():
        k = 0
        for lo in range(0, GB, chunk):
            b = k & 1
            evs[b].synchronize()
            fill(bufs[b], lo, chunk)
            with torch.cuda.stream(s):
                dev[lo:lo + chunk].copy_(bufs[b], non_blocking=True)
                evs[b].record(s)
            k += 1
        s.synchronize()
    return run


try:
    print(f"pageable, one copy: {GB / timed(one) / 1e9:.1f} GB/s", flush=True)
    for n in (2, 4, 8):
        print(f"pageable, {n} threads/streams: {GB / timed(threads(n)) / 1e9:.1f} GB/s", flush=True)
    for n in (4, 8, 16):
        print(f"pinned bounce 2x256 MiB, {n} fill threads: {GB / timed(bounce(n)) / 1e9:.1f} GB/s", flush=True)
finally:
    del m
    os.unlink(path)
