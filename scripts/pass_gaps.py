"""Where the time of one production-order pass goes (developer script): from a
rocprofv3 --kernel-trace csv of scripts/probe_inflate.py (passes without
events, phase A and phase B on their own streams), the last pass -- from its
k_bgzf_scan dispatch to the end -- split into: the time some kernel runs
(union), per kernel its own time, the time two or more kernels overlap, and
the idle gaps with the kernels on either side.
usage: python scripts/pass_gaps.py <rocprofv3 output dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    rows = []
    path = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))[-1]
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"].split("(")[0].split("<")[0].replace("hbam::", "")[:40]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == "k_bgzf_scan"]
    first = starts[-1]
    ev = rows[first:]
    t0, t1 = ev[0][0], max(e for _, e, _ in ev)
    per = defaultdict(float)
    for s, e, n in ev:
        per[n] += (e - s) / 1e6
    # sweep: busy union, overlap (>= 2 running), idle gaps
    pts = sorted([(s, 1) for s, _, _ in ev] + [(e, -1) for _, e, _ in ev])
    run, last, busy, over = 0, t0, 0, 0
    for t, d in pts:
        if run >= 1:
            busy += t - last
        if run >= 2:
            over += t - last
        run += d
        last = t
    print(f"pass {(t1 - t0) / 1e6:.3f} ms: kernels running {busy / 1e6:.3f} ms, two or more at once "
          f"{over / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms, sum of kernel times {sum(per.values()):.3f} ms")
    for n, ms in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {n:42s} {ms:8.3f} ms")
    # the largest idle gaps
    ends = sorted(ev, key=lambda r: r[1])
    gaps = []
    cur = t0
    for s, e, n in sorted(ev):
        if s > cur:
            prev = max((r for r in ev if r[1] <= s), key=lambda r: r[1], default=None)
            gaps.append(((s - cur) / 1e6, prev[2] if prev else "-", n, (cur - t0) / 1e6))
        cur = max(cur, e)
    for g, a, b, at in sorted(gaps, reverse=True)[:12]:
        print(f"  idle {g * 1e3:8.1f} us at {at:7.3f} ms: after {a} before {b}")


if __name__ == "__main__":
    main()
