"""C4 long-read probe (developer script): the C4-like BAM of bench.py's
long_read_leg through the resident device pipeline, a few passes, stage times
printed.  Run under `rocprofv3 --kernel-trace --stats` for the per-kernel
split of the record chain.
Usage: python scripts/c4_probe.py [passes]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import hbam  # noqa: E402
from hbam import synth  # noqa: E402

SEED = 0x48424D00 + 4  # bench.py long_read_leg


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    data, info = synth.make_bam(12000, mode="long", as_numpy=True, seed=SEED)
    g = hbam.Gpu(0)
    try:
        g.load(data)
        g.run()
        ts = []
        for _ in range(passes):
            t = time.perf_counter()
            g.run()
            ts.append(time.perf_counter() - t)
        st = g.run(timing=True)
    finally:
        g.close()
    dt = min(ts)
    print({"records": int(st["records"]), "U": info["uncompressed"], "C": info["compressed"],
           "blocks": info["blocks"], "best_s": round(dt, 5), "GBps_U": round(info["uncompressed"] / dt / 1e9, 2),
           "stages_ms": {k: round(st[k], 3) for k in ("ms_locate", "ms_huff", "ms_lz77", "ms_chain", "ms_decode")},
           "link_rewalks": st.get("link_rewalks"), "link_fallbacks": st.get("link_fallbacks")}, flush=True)


if __name__ == "__main__":
    main()
