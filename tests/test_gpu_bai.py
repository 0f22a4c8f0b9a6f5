"""BAI split calculator on the GPU path (hbam_get_splits_bai: the C++
BAMInputFormat::addBAISplits over the .bai's linear index, guessed starts
from the GPU BAMSplitGuesser) against the oracle restatement
(oracle/bai.py, BAMInputFormat.java:322-465)."""
import pytest

import bai
import hbam
import orc
from bai_cases import spread_bam
from test_bai import PLACEMENTS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("placement", PLACEMENTS, ids=["one", "three"])
@pytest.mark.parametrize("split_size", [60000, 150000, 400000])
def test_bai_splits_match_oracle(placement, split_size):
    data = spread_bam(6000, placement)
    b = bai.write_bai(data)
    s = orc.Stream(data)
    sp = bai.file_splits(len(data), split_size)
    want = bai.add_bai_splits(sp, s.n_ref, bai.linear_index(b), s.first_record_voff, s.guess_record_start)
    with hbam.BamFile(data) as f:
        got = f.get_splits([a for a, _ in sp], [n for _, n in sp], bai=b)
        assert got == want
        # a usable .splitting-bai wins over the .bai (addIndexedSplits first)
        sbi = f.splitting_index(4096)
        assert f.get_splits([a for a, _ in sp], [n for _, n in sp], sbi=sbi, bai=b) == \
            f.get_splits([a for a, _ in sp], [n for _, n in sp], sbi=sbi)


def test_bad_bai_is_an_error():
    data = spread_bam(2000, PLACEMENTS[0])
    with hbam.BamFile(data) as f:
        with pytest.raises(hbam.HbamError) as e:
            f.get_splits([0, 100000], [100000, len(data) - 100000], bai=b"BAM\1junk")
        assert e.value.code == hbam.E_FORMAT  # htsjdk's parse error is unchecked (not the IOException fallback)
