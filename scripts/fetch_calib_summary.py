"""FETCH_SIZE per dispatch of scripts/fetch_calib.hip (rocprofv3 --pmc FETCH_SIZE),
beside the bytes of distinct 128 B lines each dispatch touches (its stdout).
usage: python scripts/fetch_calib_summary.py <rocprofv3 out dir> <fetch_calib stdout>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    p = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(float)
    name = {}
    for r in csv.DictReader(open(p)):
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    lines = [ln for ln in open(sys.argv[2]) if ln.startswith("k_")]
    disp = [d for d in sorted(per) if name[d].startswith("k_")]
    for d, ln in zip(disp, lines):
        m = re.search(r"~?([\d.]+) lines", ln)
        touched = float(m.group(1)) * 128 if m else 0
        fb = per[d] * 1024
        print(f"{ln.strip():60s} FETCH_SIZE {fb / 1e9:7.3f} GB  line bytes {touched / 1e9:7.3f} GB  "
              f"FETCH/lines {fb / touched if touched else 0:.3f}")


if __name__ == "__main__":
    main()
