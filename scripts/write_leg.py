"""Development aid: the BGZF write path on a synthetic BAM (for rocprofv3)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import numpy as np  # noqa: E402
import hbam  # noqa: E402
from hbam import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
data, info = synth.make_bam(n, as_numpy=True)
g = hbam.Gpu(0)
g.load(data)
g.run()
g.bgzf_compress(level=5, eof=False, iters=0)
ms, nb = g.bgzf_compress(level=5, eof=False, iters=1)
same = nb == data.nbytes and bool(np.array_equal(g.fetch_compressed(0, nb), data))
print({"records": n, "ms": ms, "identical": same, "bytes": int(nb)})
