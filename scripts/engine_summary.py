"""Which DMA engine each copy took, per phase of scripts/dropin_probe2.py
(developer script).  Input: the probe's stdout and stderr in one file, run
with AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x100 (HIP's copy log: one
"HSA Copy copy_engine=0x.., dst=.., src=.., size=.., forceSDMA=.., engineType=.."
line per copy) -- the probe's MARK lines split it into phases.  Output: per
phase and per (engine, engineType), the copies and bytes, and the size
classes of the copies (the batch D2H pieces are large, the staging pieces
32 MiB).
usage: python scripts/engine_summary.py <log>"""
import re
import sys
from collections import defaultdict

PAT = re.compile(r"HSA Copy copy_engine=(0x[0-9a-fA-F]+), dst=(0x[0-9a-fA-F]+), src=(0x[0-9a-fA-F]+), "
                 r"size=(\d+), forceSDMA=(\d+), engineType=(\d+)")


def main():
    phase = "start"
    stats = defaultdict(lambda: defaultdict(lambda: [0, 0]))
    order = ["start"]
    for ln in open(sys.argv[1], errors="replace"):
        if ln.startswith("MARK "):
            phase = ln.split()[1]
            if phase not in order:
                order.append(phase)
            continue
        if ln.startswith(("mapped", "resident")):
            print(ln.rstrip()[:200])
        m = PAT.search(ln)
        if not m:
            continue
        eng, dst, src, size, force, etype = m.groups()
        size = int(size)
        cls = "big" if size >= (64 << 20) else "32M" if size >= (16 << 20) else "small"
        e = stats[phase][(eng, etype, cls)]
        e[0] += 1
        e[1] += size
    if not stats:  # no copy line in the expected format: show what the log holds about copies
        from collections import Counter
        seen = Counter()
        for ln in open(sys.argv[1], errors="replace"):
            if "opy" in ln or "SDMA" in ln or "engine" in ln:
                seen[re.sub(r"0x[0-9a-fA-F]+|\d+", "#", ln.strip())[:160]] += 1
        print("no 'HSA Copy copy_engine=' lines; most common copy-related line shapes:")
        for shape, n in seen.most_common(25):
            print(f"  {n:7d}  {shape}")
    for ph in order:
        if ph not in stats:
            continue
        print(f"== {ph}")
        for (eng, etype, cls), (n, b) in sorted(stats[ph].items()):
            print(f"   engine {eng} type {etype} {cls:5s}: {n:6d} copies {b / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
