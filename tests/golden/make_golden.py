"""Regenerate tests/golden/ (run in the build container; /root/reference is
not available on the GPU box).

Inputs are data fixtures the reference's own tests hold
(/root/reference/src/test/resources: test.bam, HiSeq.10000.vcf.bgzf.gz,
test.vcf.bgzf.gz, test.bgzf.bcf; MIT, LICENSE.txt).  Expected outputs come from
the C oracle (oracle/hbam_oracle.c), cross-checked against the independent
Python restatement (oracle/py_oracle.py) and against the pins the reference
tests assert:
  TestBAMSplitGuesser.java:21   first record voff of test.bam
  TestBGZFSplitGuesser.java:36  BGZF boundaries 821/821 and 16688/509222
  TestSplittingBAMIndexer.java  bamSize() == file length
Plain-text twins of the BGZF fixtures pin inflate (stored here as sha256).
"""
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import orc  # noqa: E402
import py_oracle  # noqa: E402

RES = "/root/reference/src/test/resources"


def main():
    for f in ("test.bam", "HiSeq.10000.vcf.bgzf.gz", "test.vcf.bgzf.gz", "test.bgzf.bcf"):
        shutil.copyfile(os.path.join(RES, f), os.path.join(HERE, f))
    bam = open(os.path.join(HERE, "test.bam"), "rb").read()
    s = orc.Stream(bam)
    rc, r = s.decode_all()
    assert rc == 0 and len(r["key"]) == 2277
    # independent cross-check
    pr = py_oracle.records(bam)
    assert [v for v, _ in pr] == [int(x) for x in r["voff"]]
    assert [k for _, k in pr] == [int(x) for x in r["key"]]
    assert s.first_record_voff == 0x196A  # TestBAMSplitGuesser pin (restated)
    np.savez(os.path.join(HERE, "test.bam.records.npz"), **r)
    meta = {"first_record_voff": s.first_record_voff, "n_ref": s.n_ref, "header_end": s.header_end,
            "n_records": int(len(r["key"])), "file_size": len(bam),
            "blocks": [[int(b["coff"]), int(b["csize"]), int(b["isize"]), int(b["ustart"])] for b in s.blocks],
            "inflated_sha256": hashlib.sha256(s.data).hexdigest(), "inflated_len": len(s.data)}
    for g in (1, 2, 10, 4096):
        idx = s.splitting_index(g)
        assert idx == py_oracle.splitting_index(bam, g)
        assert int.from_bytes(idx[-8:], "big") >> 16 == len(bam)
        open(os.path.join(HERE, f"test.bam.g{g}.splitting-bai"), "wb").write(idx)
    # guesser at every block start and just before it
    guesses = []
    for b in s.blocks[1:]:
        c = int(b["coff"])
        for beg in (c, c - 5, c + 1):
            end = beg + 3 * 0xFFFF + 0xFFFE
            guesses.append([beg, end, s.guess_record_start(beg, end)])
    for beg in range(1000, len(bam), 7919):
        end = min(len(bam), beg + 40000)
        guesses.append([beg, end, s.guess_record_start(beg, end)])
    meta["guesses"] = guesses
    # split planning (SPLIT_MAXSIZE-style byte ranges) with and without the index
    plans = []
    for split in (40000, 65536, 100000):
        starts = list(range(0, len(bam), split))
        lengths = [min(split, len(bam) - x) for x in starts]
        sbi = s.splitting_index(4096)
        plans.append({"split": split, "starts": starts, "lengths": lengths,
                      "indexed": s.get_splits(starts, lengths, sbi),
                      "probabilistic": s.get_splits(starts, lengths, None)})
    meta["plans"] = plans
    # BGZF text fixtures: inflate known answers + block discovery pins
    text = {}
    for f, plain in (("HiSeq.10000.vcf.bgzf.gz", "HiSeq.10000.vcf"), ("test.vcf.bgzf.gz", "test.vcf"),
                     ("test.bgzf.bcf", "test.uncompressed.bcf")):
        data = open(os.path.join(HERE, f), "rb").read()
        x = orc.Stream(data, check_crc=True, parse_header=False)
        want = open(os.path.join(RES, plain), "rb").read()
        assert x.data == want
        bnd, start = [], 1
        while True:
            ns = orc.guess_next_bgzf_block_start(data, start, len(data))
            if ns == len(data):
                break
            bnd.append(ns)
            start = ns + 1
        text[f] = {"sha256": hashlib.sha256(want).hexdigest(), "len": len(want),
                   "coffs": [int(b["coff"]) for b in x.blocks], "boundaries": bnd}
    assert text["test.vcf.bgzf.gz"]["boundaries"][0] == 821
    assert text["HiSeq.10000.vcf.bgzf.gz"]["boundaries"][0] == 16688
    assert text["HiSeq.10000.vcf.bgzf.gz"]["boundaries"][-1] == 509222
    meta["bgzf_text"] = text
    json.dump(meta, open(os.path.join(HERE, "golden.json"), "w"), indent=1)
    print("golden written:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
