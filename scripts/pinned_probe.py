"""C2 end-to-end from page-locked host memory (bench.py pinned_host_leg) on its
own, for a rocprofv3 kernel + memory-copy trace (developer probe).
usage: python scripts/pinned_probe.py [records] [piece MiB]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import hbam  # noqa: E402
from hbam import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    piece = (int(sys.argv[2]) if len(sys.argv) > 2 else 256) << 20
    data, info = synth.make_bam(n, as_numpy=True)
    g = hbam.Gpu(0)
    try:
        with hbam.PinnedBuffer(data.nbytes) as buf:
            buf.array[:] = data
            g.load(data)
            g.run_streamed(buf.ptr, buf.nbytes, piece)
            for _ in range(3):
                t = time.perf_counter()
                st = g.run_streamed(buf.ptr, buf.nbytes, piece)
                dt = time.perf_counter() - t
                print(f"streamed: {dt * 1e3:.1f} ms {info['uncompressed'] / dt / 1e9:.1f} GB/s U, "
                      f"{data.nbytes / dt / 1e9:.1f} GB/s C, records {st['records']}", flush=True)
            t = time.perf_counter()
            g.run()
            print(f"resident pass {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    finally:
        g.close()


if __name__ == "__main__":
    main()
