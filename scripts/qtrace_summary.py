"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace CSV run of
scripts/dropin_probe2.py (gpu_round.sh qtrace): for every `mapped<rep>` window
the probe marked, each kernel's hardware queue(s), count and mean duration,
and the copies by direction (count, mean duration, rate).
usage: python scripts/qtrace_summary.py <out dir holding qtrace/ and qtrace.log>"""
import collections
import csv
import glob
import json
import os
import re
import sys


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as fh:
            out.extend(csv.DictReader(fh))
    return out


def col(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    return None


def main():
    d = sys.argv[1]
    marks = {}
    for line in open(os.path.join(d, "qtrace.log")):
        m = re.match(r"MARK (\S+) mono=(\d+) boot=(\d+)", line)
        if m:
            marks[m.group(1)] = (int(m.group(2)), int(m.group(3)))
    kern = rows(os.path.join(d, "qtrace", "**", "*kernel_trace.csv"))
    copy = rows(os.path.join(d, "qtrace", "**", "*memory_copy_trace.csv"))
    if not kern:
        sys.exit("no kernel trace")
    t0 = min(int(r["Start_Timestamp"]) for r in kern)
    t1 = max(int(r["End_Timestamp"]) for r in kern)
    # the clock whose markers fall inside the trace's span
    clock = 0
    for c in (0, 1):
        if all(t0 - 60e9 < v[c] < t1 + 60e9 for v in marks.values()):
            clock = c
            break
    reps = sorted({k[:-6] for k in marks if k.endswith("_begin")})
    out = {"clock": ("monotonic", "boottime")[clock], "columns": {"kernel": list(kern[0].keys()),
                                                               "copy": list(copy[0].keys()) if copy else []}}
    for rep in reps:
        b, e = marks[rep + "_begin"][clock], marks[rep + "_end"][clock]
        ks = collections.defaultdict(lambda: {"n": 0, "ns": 0, "queues": collections.Counter(),
                                              "streams": collections.Counter()})
        for r in kern:
            s = int(r["Start_Timestamp"])
            if b <= s <= e:
                name = r["Kernel_Name"].split("(")[0][:60]
                k = ks[name]
                k["n"] += 1
                k["ns"] += int(r["End_Timestamp"]) - s
                k["queues"][col(r, "Queue_Id", "Queue_ID") or "?"] += 1
                k["streams"][col(r, "Stream_Id", "Stream_ID") or "?"] += 1
        cs = collections.defaultdict(lambda: {"n": 0, "ns": 0, "bytes": 0, "streams": collections.Counter()})
        for r in copy:
            s = int(r["Start_Timestamp"])
            if b <= s <= e:
                c = cs[col(r, "Direction", "Kind") or "?"]
                c["n"] += 1
                c["ns"] += int(r["End_Timestamp"]) - s
                c["bytes"] += int(col(r, "Bytes", "Size", "Copy_Bytes") or 0)
                c["streams"][col(r, "Stream_Id", "Stream_ID") or "?"] += 1
        # the copies' own timeline: time each direction is in flight, time both
        # are, and each direction's rate alone vs beside the other
        iv = collections.defaultdict(list)
        for r in copy:
            s0 = int(r["Start_Timestamp"])
            if b <= s0 <= e:
                iv[col(r, "Direction", "Kind") or "?"].append((s0, int(r["End_Timestamp"]),
                                                               int(col(r, "Bytes", "Size", "Copy_Bytes") or 0)))
        out_ov = {}
        dirs = sorted(iv)
        if len(dirs) >= 2:
            ev = sorted([(s0, 1, d) for d in dirs for s0, _, _ in iv[d]] + [(e0, -1, d) for d in dirs for _, e0, _ in iv[d]])
            run = collections.Counter()
            last = ev[0][0] if ev else 0
            acc = collections.Counter()
            for t, dd, d in ev:
                act = tuple(x for x in dirs if run[x] > 0)
                acc[act] += t - last
                run[d] += dd
                last = t
            out_ov["ms_active"] = {"+".join(k) if k else "none": round(v / 1e6, 2) for k, v in acc.items()}
            for d in dirs:
                others = [x for o in dirs if o != d for x in iv[o]]
                alone = [0, 0]
                beside = [0, 0]
                for s0, e0, nb in iv[d]:
                    hit = any(os_ < e0 and oe > s0 for os_, oe, _ in others)
                    tgt = beside if hit else alone
                    tgt[0] += nb
                    tgt[1] += e0 - s0
                out_ov[d] = {"GBps_alone": round(alone[0] / alone[1], 2) if alone[1] else None,
                             "GBps_beside_other": round(beside[0] / beside[1], 2) if beside[1] else None,
                             "GB_alone": round(alone[0] / 1e9, 3), "GB_beside": round(beside[0] / 1e9, 3)}
        out[rep] = {
            "overlap": out_ov,
            "seconds": round((e - b) / 1e9, 4),
            "kernels": {n: {"n": v["n"], "mean_us": round(v["ns"] / v["n"] / 1e3, 1), "queues": dict(v["queues"]),
                            "streams": dict(v["streams"])} for n, v in sorted(ks.items(), key=lambda x: -x[1]["ns"])},
            "copies": {n: {"n": v["n"], "mean_us": round(v["ns"] / v["n"] / 1e3, 1),
                           "GBps": round(v["bytes"] / max(v["ns"], 1), 2) if v["bytes"] else None,
                           "streams": dict(v["streams"])} for n, v in cs.items()},
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
