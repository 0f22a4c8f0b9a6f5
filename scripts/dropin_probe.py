"""Where the drop-in call's time goes (hbam_open(path) + hbam_decode_span in
1M-record batches into pinned host memory) on a C2-shaped file.
usage: python scripts/dropin_probe.py [records]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import hbam
from hbam import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
data, info = synth.make_bam(n, as_numpy=True)
path = "/dev/shm/hbam_dropin_probe.bam"
data.tofile(path)
del data
ALL = (1 << 64) - 1
try:
    for window, batch in ((0, 1 << 16), (0, 1 << 18), (0, 1 << 20), (64 << 20, 1 << 20), (128 << 20, 1 << 20),
                          (512 << 20, 1 << 20), (0, 1 << 20)):
        t0 = time.perf_counter()
        with hbam.BamFile(path=path, window_bytes=window) as f:
            first = f.header()["first_record_voff"]
            t1 = time.perf_counter()
            r = f.scan_batches(first, ALL, batch)
            t2 = time.perf_counter()
            u = f.file_stats()[1]
        print(f"window {window >> 20} MiB batch {batch}: open+header {t1 - t0:.3f}s scan {t2 - t1:.3f}s total {u / (t2 - t0) / 1e9:.1f} GB/s "
              f"({r[1]} batches)", flush=True)
    for rep in range(2):
        t0 = time.perf_counter()
        with hbam.BamFile(path=path) as f:
            t1 = time.perf_counter()
            first = f.header()["first_record_voff"]
            t2 = time.perf_counter()
            r1 = f.scan_batches(first, ALL, 1 << 20)
            t3 = time.perf_counter()
            r2 = f.scan_batches(first, ALL, 1 << 20)
            t4 = time.perf_counter()
            t5 = time.perf_counter()
            f.prefetch(0, f.size)
            t6 = time.perf_counter()
            r3 = f.scan_batches(first, ALL, 1 << 20)
            t7 = time.perf_counter()
            u = f.file_stats()[1]
        print(f"rep {rep}: open {t1 - t0:.3f}s header {t2 - t1:.3f}s scan1 {t3 - t2:.3f}s ({u / (t3 - t2) / 1e9:.1f} GB/s) "
              f"scan2 {t4 - t3:.3f}s ({u / (t4 - t3) / 1e9:.1f} GB/s) prefetch {t6 - t5:.3f}s "
              f"scan_resident {t7 - t6:.3f}s ({u / (t7 - t6) / 1e9:.1f} GB/s) records {r1[0]} {r2[0]} {r3[0]}", flush=True)
finally:
    os.unlink(path)
