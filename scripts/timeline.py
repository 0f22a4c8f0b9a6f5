"""Merged kernel + memory-copy timeline from a rocprofv3 csv run (developer
script).  usage: python scripts/timeline.py <dir>/<prefix> [t0_ms] [t1_ms]
prints one line per dispatch/copy: start ms, duration ms, stream, queue, name."""
import csv
import sys


def rows(prefix):
    out = []
    with open(prefix + "_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"], "q" + r["Queue_Id"],
                        r["Kernel_Name"].split("(")[0][:48]))
    try:
        with open(prefix + "_memory_copy_trace.csv") as f:
            for r in csv.DictReader(f):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s" + r["Stream_Id"], "dma",
                            r["Direction"].replace("MEMORY_COPY_", "")))
    except FileNotFoundError:
        pass
    return sorted(out)


def main():
    ev = rows(sys.argv[1])
    base = ev[0][0]
    t0 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    t1 = float(sys.argv[3]) if len(sys.argv) > 3 else 1e18
    for s, e, st, q, name in ev:
        ms = (s - base) / 1e6
        if t0 <= ms <= t1:
            print(f"{ms:10.3f} {(e - s) / 1e6:8.3f} {st:>4} {q:>4} {name}")


if __name__ == "__main__":
    main()
