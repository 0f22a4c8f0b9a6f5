"""BAI split calculator (BAMInputFormat.addBAISplits, BAMInputFormat.java:322-465)
on CPU: the oracle restatement (oracle/bai.py) plans splits that cover every
record exactly once, and the .bai reader/writer round-trip.  The GPU planner
is compared with it in test_gpu_bai.py.

Parity with the reference is unpinned beyond the restatement: its tests
(TestBAMInputFormat.testMultipleSplitsBaiEnabled*: 3 splits of 1080/524/398
records) run on a BAM and .bai that htsjdk writes at test time
(BAMTestUtil.writeBamFile), which cannot be produced here."""
import pytest

import bai
import orc
from bai_cases import spread_bam

PLACEMENTS = [
    [(0, 10000, 40)],                                  # one contig, ~25 windows
    [(1, 5000, 300), (4, 0, 500), (7, 2000000, 90)],  # empty contigs between, a gap of windows
]


def _plan(data, split_size):
    s = orc.Stream(data)
    idx = bai.linear_index(bai.write_bai(data))
    sp = bai.file_splits(len(data), split_size)
    return s, sp, bai.add_bai_splits(sp, s.n_ref, idx, s.first_record_voff, s.guess_record_start)


@pytest.mark.parametrize("placement", PLACEMENTS, ids=["one", "three"])
@pytest.mark.parametrize("split_size", [60000, 150000, 400000])
def test_oracle_bai_splits_cover_every_record_once(placement, split_size):
    data = spread_bam(6000, placement)
    s, sp, plan = _plan(data, split_size)
    assert len(plan) == len(sp)
    rc, want = s.decode_all()
    got = []
    for a, e in plan:
        rc, r = s.decode_span(a, e)
        assert rc == 0
        got += [int(v) for v in r["voff"]]
    assert got == [int(v) for v in want["voff"]]


def test_linear_index_roundtrip():
    data = spread_bam(3000, PLACEMENTS[1])
    b = bai.write_bai(data)
    li = bai.linear_index(b)
    assert [bool(x) for x in li[:8]] == [False, True, False, False, True, False, False, True]
    assert all(li[1][k] <= li[1][k + 1] for k in range(len(li[1]) - 1))
    with pytest.raises(ValueError):
        bai.linear_index(b"BAM\1" + b[4:])


def test_oracle_bai_splits_guess_a_start():
    """A split no linear entry starts in gets BAMSplitGuesser's start and cuts
    the split before it (:432-444)."""
    data = spread_bam(6000, PLACEMENTS[0])
    s = orc.Stream(data)
    idx = bai.linear_index(bai.write_bai(data))
    calls = []

    def guess(a, e):
        calls.append(a)
        return s.guess_record_start(a, e)

    plan = bai.add_bai_splits(bai.file_splits(len(data), 60000), s.n_ref, idx, s.first_record_voff, guess)
    assert calls
    starts = {a for a, _ in plan}
    assert all(s.guess_record_start(a, a + 60000) in starts for a in calls)
