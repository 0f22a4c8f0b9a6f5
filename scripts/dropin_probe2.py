"""Per-batch timing of the drop-in call (developer probe): hbam_decode_span in 1M-record
batches from the mapped file and from a resident copy, every batch timed.
usage: python scripts/dropin_probe2.py [records]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import hbam  # noqa: E402
from hbam import synth  # noqa: E402

ALL = (1 << 64) - 1


def link_rates():
    import torch
    n = 1 << 32
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out[name] = round(3 * n / (time.perf_counter() - t) / 1e9, 1)
    del h, d
    torch.cuda.empty_cache()
    return out


def batches(f, first, nrec):
    b = hbam.Batch()
    v, ts, n = first, [], 0
    import ctypes as C
    while True:
        t = time.perf_counter()
        rc = hbam._L.hbam_decode_span(f._h, v, ALL, nrec, C.byref(b))
        ts.append(round((time.perf_counter() - t) * 1e3, 1))
        if rc != 0 or b.n == 0:
            break
        n += b.n
        v = b.next_voff
    return n, ts


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    data, info = synth.make_bam(n, as_numpy=True)
    path = "/dev/shm/hbam_dropin_probe2.bam"
    data.tofile(path)
    del data
    try:
        for rep in range(2):
            with hbam.BamFile(path=path) as f:
                first = f.header()["first_record_voff"]
                t = time.perf_counter()
                m, ts = batches(f, first, 1 << 20)
                dt = time.perf_counter() - t
                print(f"mapped rep {rep}: {m} records {dt:.3f}s {info['uncompressed'] / dt / 1e9:.1f} GB/s batches ms {ts}",
                      flush=True)
                f.prefetch(0, f.size)
                t = time.perf_counter()
                m, ts = batches(f, first, 1 << 20)
                dt = time.perf_counter() - t
                print(f"resident rep {rep}: {dt:.3f}s {info['uncompressed'] / dt / 1e9:.1f} GB/s batches ms {ts}",
                      flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
