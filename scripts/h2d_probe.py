"""Host->HBM rates on the box: pinned reload (SDMA), streamed pass (copy kernel + inflate)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import numpy as np
import hbam
from hbam import synth
data, info = synth.make_bam(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, as_numpy=True)
g = hbam.Gpu(0)
g.load(data)
with hbam.PinnedBuffer(data.nbytes) as buf:
    buf.array[:] = data
    for _ in range(2):
        ms = g.reload(buf.ptr, buf.nbytes, pinned=False)
    print(f"reload from page-locked memory: {ms:.1f} ms = {data.nbytes / ms / 1e6:.1f} GB/s")
    g.run()
    for piece in (16 << 20, 64 << 20, 256 << 20):
        g.run_streamed(buf.ptr, buf.nbytes, piece)
        t = time.perf_counter()
        st = g.run_streamed(buf.ptr, buf.nbytes, piece)
        dt = time.perf_counter() - t
        print(f"streamed piece {piece >> 20} MiB: {dt * 1e3:.1f} ms wall, ms_total {st['ms_total']:.1f}, "
              f"{info['uncompressed'] / dt / 1e9:.1f} GB/s U", flush=True)
    t = time.perf_counter()
    st = g.run(timing=False)
    print(f"resident run: {(time.perf_counter() - t) * 1e3:.1f} ms")
g.close()
