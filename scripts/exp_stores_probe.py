"""Phase-A time with scattered (default) vs coalesced emit stores
(scripts/exp_stores_patch.py build): one normal pass, then timing passes
with HBAM_EXP_SKIPB set (phase B skipped, the emit's stores to fixed slots).
usage: HBAM_LIB=... python scripts/exp_stores_probe.py [records]"""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    import hbam
    from hbam import synth
    data, _ = synth.make_bam(n, as_numpy=True)
    g = hbam.Gpu(0)
    g.load(data)
    res = {}
    for mode in ("normal", "coalesced", "normal2"):
        if mode == "coalesced":
            os.environ["HBAM_EXP_SKIPB"] = "1"
        else:
            os.environ.pop("HBAM_EXP_SKIPB", None)
        best = None
        for _ in range(4):
            st = g.run(timing=True)
            if best is None or st["ms_huff"] < best["ms_huff"]:
                best = st
        res[mode] = {k: round(v, 3) for k, v in best.items() if k in ("ms_huff", "ms_lz77", "ms_tables", "ms_total")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
