"""Sharded read through the GPU decoder (hbam.BamFile on cuda:0 in every rank,
gloo for the metadata all_gathers -- one GPU box): same checks as
test_shard.py, against the oracle."""
import pytest

from hbam import synth
from test_shard import check_against_oracle, run_sharded

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,g,kw", [
    (2, 4096, dict(n_records=20000)),
    (3, 7, dict(n_records=4000, block_payload=4096)),
    (2, 3, dict(n_records=30, mode="long")),
])
def test_gpu_sharded_read_matches_whole_file(tmp_path, world, g, kw):
    data, _ = synth.make_bam(**kw)
    parts = run_sharded(data, world, g, tmp_path, use_gpu=True)
    check_against_oracle(data, parts, g)
