"""Loops of one kernel in a hipcc -S listing (developer script): every
backward branch [label, branch], its size, and the scratch (spill) and LDS
instructions inside -- to see whether spills land in a hot loop.
usage: python scripts/isa_loops.py <file.s> <kernel symbol substring> [min alignbit]"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    min_ab = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name) or (name in l and l.split(";")[0].strip().endswith(":") and l.startswith("_Z")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB[\w_]+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB[\w_]+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            a = labels[m.group(2)]
            seg = body[a:i + 1]
            n_ins = sum(1 for x in seg if x.startswith("\t") and not x.strip().startswith((";", ".")))
            sc = sum(1 for x in seg if "scratch_" in x)
            ab = sum(1 for x in seg if "v_alignbit" in x)
            ds = sum(1 for x in seg if re.search(r"\bds_(read|load)", x))
            if ab >= min_ab:
                loops.append((a, i, n_ins, sc, ab, ds))
    for a, i, n, sc, ab, ds in loops:
        print(f"loop lines {a + start + 1}-{i + start + 1}: {n} instrs, scratch {sc}, alignbit {ab}, ds_read {ds}")


if __name__ == "__main__":
    main()
