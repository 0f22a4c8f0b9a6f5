"""Sharded read through the GPU decoder (hbam.BamFile on cuda:0 in every rank,
gloo for the metadata all_gathers -- one GPU box): same checks as
test_shard.py, against the oracle."""
import pytest

from hbam import synth
from test_shard import GUESS_BYTES, WINDOW, check_against_oracle, check_rank_local_reads, run_sharded

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,g,kw", [
    (2, 4096, dict(n_records=40000)),
    (4, 7, dict(n_records=30000, block_payload=4096)),
    (3, 3, dict(n_records=60, mode="long")),
])
def test_gpu_sharded_read_matches_whole_file(tmp_path, world, g, kw):
    """Each rank opens the file by path (split-local) and decodes its split
    in windows: same records / index as the oracle over the whole file, and
    each rank copies about its own byte range to HBM (header window + guesser
    window + its split + the window that finishes its last record)."""
    data, _ = synth.make_bam(**kw)
    parts = run_sharded(data, world, g, tmp_path, use_gpu=True)
    check_against_oracle(data, parts, g)
    check_rank_local_reads(data, parts, min(WINDOW, 1 << 20) + GUESS_BYTES + 2 * 65536 + 2 * WINDOW)
