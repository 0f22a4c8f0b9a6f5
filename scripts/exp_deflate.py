"""Time the GPU BGZF compressor on a synthetic BAM's inflated stream and check
the recompressed bytes equal the file (zlib level 5, fresh stream per block)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import numpy as np
import hbam
from hbam import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
data, info = synth.make_bam(n, seed=0x48424D00, as_numpy=True)
print(info, flush=True)
g = hbam.Gpu(0)
g.load(data)
g.run()
t = time.perf_counter()
ms, nb = g.bgzf_compress(level=5, eof=False, iters=0)
print(f"first call {time.perf_counter()-t:.3f}s  ms={ms:.2f}", flush=True)
ms, nb = g.bgzf_compress(level=5, eof=False, iters=2)
got = g.fetch_compressed(0, nb)
print(f"blocks {info['blocks']} U {info['uncompressed']} -> {nb} bytes, {ms:.2f} ms/pass, "
      f"{info['uncompressed']/ms/1e6:.2f} GB/s payload, identical={nb == data.nbytes and np.array_equal(got, data)}", flush=True)
