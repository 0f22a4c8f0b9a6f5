"""PCIe duplex probe (developer): pinned host<->HBM copy rates one direction at a
time and both at once on two streams (does a host->HBM copy slow a concurrent
HBM->host copy?).  usage: python scripts/duplex_probe.py [GiB]"""
import sys
import time

import torch


def main():
    n = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 1 << 30
    hs = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    hd = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    ds = torch.empty(n, dtype=torch.uint8, device="cuda")
    dd = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            ds.copy_(hs, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            hd.copy_(dd, non_blocking=True)

    def timed(fns, reps=3):
        for f in fns:
            f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            for f in fns:
                f()
        torch.cuda.synchronize()
        return reps * n / (time.perf_counter() - t) / 1e9

    print("h2d alone %.1f GB/s" % timed([h2d]))
    print("d2h alone %.1f GB/s" % timed([d2h]))
    b = timed([h2d, d2h])
    print("both at once: %.1f GB/s each direction (%.1f GB/s total)" % (b, 2 * b))
    # d2h timed with a smaller h2d beside it (as the drop-in: 1.4 GB staged against 3.6 GB of batches)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    with torch.cuda.stream(s2):
        ev[0].record()
        hd.copy_(dd, non_blocking=True)
        ev[1].record()
    with torch.cuda.stream(s1):
        ds[: n // 3].copy_(hs[: n // 3], non_blocking=True)
    torch.cuda.synchronize()
    print("d2h beside a third-size h2d: %.1f GB/s" % (n / ev[0].elapsed_time(ev[1]) / 1e6))
    if "--kernel" not in sys.argv:
        return
    import ctypes
    import os
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_duplex.so"))
    lib.duplex_pull.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    for blocks in (32, 64, 128, 256, 1024):
        def pull():
            rc = lib.duplex_pull(hs.data_ptr(), ds.data_ptr(), n, blocks, s1.cuda_stream)
            assert rc == 0, rc
        r = timed([pull])
        torch.cuda.synchronize()
        assert torch.equal(ds[:4096].cpu(), hs[:4096]), "pull copied wrong bytes"
        b = timed([pull, d2h])
        print("kernel h2d, %4d blocks: alone %.1f GB/s; beside an SDMA d2h %.1f GB/s each (%.1f total)"
              % (blocks, r, b, 2 * b))


if __name__ == "__main__":
    main()
