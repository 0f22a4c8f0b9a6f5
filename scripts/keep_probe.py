"""Small decodes through a chosen libhbam.so (HBAM_LIB) with their results
against the oracle (developer script for phase-A changes).
usage: HBAM_LIB=... python scripts/keep_probe.py [records]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    import hbam
    from hbam import synth
    data, info = synth.make_bam(n, as_numpy=True)
    print("file", data.nbytes, flush=True)
    g = hbam.Gpu(0)
    t = time.time()
    g.load(data)
    print("load ok %.2fs" % (time.time() - t), flush=True)
    st = g.run(timing=True)
    print("run ok", {k: round(v, 3) for k, v in st.items() if k.startswith("ms_")}, flush=True)
    g.close()


if __name__ == "__main__":
    main()
