import sys, os, ctypes as C
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import numpy as np, hbam
from hbam import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
data, info = synth.make_bam(n, as_numpy=True)
g = hbam.Gpu(0); g.load(data); g.run()
L = hbam._L
L.hbam_probe_read.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(32, np.uint64)
L.hbam_probe_read(buf.ctypes.data, 1)
st = g.run(timing=True)
L.hbam_probe_read(buf.ctypes.data, 1)
print(info, {k: round(st[k], 2) for k in ("ms_huff", "ms_lz77", "ms_total")})
nA, nB = int(buf[15]), int(buf[16])
names = {0: "A stage", 1: "A hdr(wave0)+barrier", 3: "A spec", 4: "A sync loop", 5: "A scan", 6: "A emit", 7: "A total",
         17: "B sum", 18: "B fill", 19: "B resolve", 20: "B store", 21: "B total"}
print("A WGs", nA, "deflate blocks", int(buf[2]), "per BGZF", int(buf[2]) / max(nA, 1), "sync iters/defl", int(buf[8]) / max(int(buf[2]), 1))
for i, nm in names.items():
    d = nA if i < 16 else nB
    print(f"{nm:24s} {int(buf[i]) / max(d, 1):12.0f} cycles/WG")
print("sync re-decodes", int(buf[12]), "non-merge", int(buf[9]), "merge", int(buf[10]), "non-merge with spec tokens", int(buf[11]))
