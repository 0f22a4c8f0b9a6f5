"""BGZFSplitGuesser.guessNextBGZFBlockStart on the GPU (util/BGZFSplitGuesser.java:64-112;
the split search of the BGZF text formats), against the reference's own pins
(TestBGZFSplitGuesser.java:36-37) and the oracle at random split points."""
import numpy as np
import pytest

import hbam
import orc
from conftest import golden_path
from hbam import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,first,last", [("test.vcf.bgzf.gz", 821, 821),
                                             ("HiSeq.10000.vcf.bgzf.gz", 16688, 509222)])
def test_reference_pins(name, first, last):
    data = open(golden_path(name), "rb").read()
    with hbam.BamFile(data, bam=False) as f:
        bnd, start = [], 1
        while True:  # TestBGZFSplitGuesser.test loop, one split point at a time
            ns = f.guess_bgzf_block_starts([start], [len(data)])[0]
            if ns == len(data):
                break
            bnd.append(ns)
            start = ns + 1
        # and every split point of that walk in one batched launch
        begs = [1] + [b + 1 for b in bnd]
        assert f.guess_bgzf_block_starts(begs, [len(data)] * len(begs)) == bnd + [len(data)]
    assert bnd[0] == first and bnd[-1] == last


@pytest.mark.parametrize("src", ["HiSeq.10000.vcf.bgzf.gz", "test.bgzf.bcf", "synthetic_bam"])
def test_random_split_points_vs_oracle(src):
    if src == "synthetic_bam":
        data, _ = synth.make_bam(20000, seed=0x42475A47)
        bam = True
    else:
        data = open(golden_path(src), "rb").read()
        bam = False
    rng = np.random.default_rng(7)
    n = len(data)
    begs = sorted(set(int(x) for x in rng.integers(0, n, 300)))
    ends = [min(n, b + int(w)) for b, w in zip(begs, rng.integers(1, 200000, len(begs)))]
    ends[::7] = [n] * len(ends[::7])
    want = [orc.guess_next_bgzf_block_start(data, b, e) for b, e in zip(begs, ends)]
    with hbam.BamFile(data, bam=bam) as f:
        got = f.guess_bgzf_block_starts(begs, ends)
    assert got == want
