"""Stage times of one resident pass over a synthetic C2-shaped BAM.

usage: python scripts/probe_inflate.py [records] [lib.so ...]
Each extra argument is an alternative libhbam.so (HBAM_LIB) run in its own
child process on the same file, so variants compare on identical input.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))


def one(n, reps=5):
    import numpy as np
    import hbam
    from hbam import synth
    data, info = synth.make_bam(n, as_numpy=True)
    g = hbam.Gpu(0)
    g.load(data)
    best = None
    for _ in range(reps + 1):
        try:
            st = g.run(timing=True)
        except hbam.HbamError as e:  # cut variants (stage timing only)
            st = {"ms_total": 0.0, "error": 1.0}
        if best is None or st["ms_total"] < best["ms_total"]:
            best = st
    out = {k: round(v, 3) for k, v in best.items() if k.startswith("ms_")}
    # the production order (phase A / phase B overlapped on two streams, no
    # events), wall clock per pass, best of 3 groups of 5
    import time
    walls = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(5):
            g.run(timing=False)
        walls.append((time.perf_counter() - t) / 5 * 1e3)
    out["wall_ms_overlapped"] = round(min(walls), 3)
    out["records"] = n
    out["lib"] = os.environ.get("HBAM_LIB", "default")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    libs = sys.argv[2:]
    if os.environ.get("HBAM_PROBE_CHILD") or not libs:
        one(n)
    else:
        for lib in libs:
            env = dict(os.environ, HBAM_LIB=os.path.abspath(lib), HBAM_PROBE_CHILD="1")
            subprocess.run([sys.executable, __file__, str(n)], env=env, check=True, timeout=300)
