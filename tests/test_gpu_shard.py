"""Sharded read through the GPU decoder (hbam.BamFile on cuda:0 in every rank,
gloo for the metadata all_gathers -- one GPU box): same checks as
test_shard.py, against the oracle."""
import os

import pytest

from hbam import synth
from test_shard import GUESS_BYTES, WINDOW, check_against_oracle, check_rank_local_reads, run_sharded

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,g,kw", [
    (2, 4096, dict(n_records=40000)),
    (4, 7, dict(n_records=30000, block_payload=4096)),
    (3, 3, dict(n_records=60, mode="long")),
    (8, 4096, dict(n_records=120000)),                   # the 8-GPU node's rank count (all on cuda:0)
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


def _strong_worker(rank, world, port, path, outdir, granularity):
    """bench.py's C3 sequence per rank: split, device decode with digests,
    counts -> global ordinals, hbam_splitting_entries of the split."""
    import numpy as np
    import torch.distributed as dist
    import hbam
    from hbam import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def all_gather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    with hbam.BamFile(path=path, device=0, window_bytes=WINDOW) as f:
        first = f.header()["first_record_voff"]
        split = shard.ShardedBamReader(f, os.path.getsize(path), first, rank, world, all_gather).split()
        if split is None:
            mine, ent = (0, 0, 0), np.zeros(0, np.uint64)
            all_gather(mine)
        else:
            st = f.decode_span_device(*split, digest=True)
            mine = (st["records"], st["key_digest"], st["voff_digest"])
            counts = all_gather(mine)
            base = sum(c[0] for c in counts[:rank])
            n, ent = f.splitting_entries(*split, granularity, base)
            assert n == mine[0], (n, mine)
    np.savez(os.path.join(outdir, f"s{rank}.npz"), mine=np.array(mine, np.uint64), ent=ent)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,g,kw", [
    (3, 4096, dict(n_records=50000)),
    (4, 5, dict(n_records=20000, block_payload=4096)),
    (2, 2, dict(n_records=40, mode="long")),
    (8, 4096, dict(n_records=120000, mode="wgs")),       # 8 ranks over C3's model
])
def test_gpu_strong_split_digests_and_index(tmp_path, world, g, kw):
    """One file split over the ranks (bench.py --workload c3): the ranks'
    order-sensitive digests compose to the oracle's whole-file digests and
    their hbam_splitting_entries, concatenated between the first record's
    voff and size << 16, are the oracle's .splitting-bai byte for byte."""
    import numpy as np
    import orc
    from hbam import shard
    from test_shard import _free_port
    import torch.multiprocessing as mp
    data, _ = synth.make_bam(**kw)
    path = os.path.join(tmp_path, "in.bam")
    open(path, "wb").write(data)
    mp.spawn(_strong_worker, args=(world, _free_port(), path, str(tmp_path), g), nprocs=world, join=True)
    parts = [np.load(os.path.join(tmp_path, f"s{r}.npz")) for r in range(world)]
    n, kd = orc.digest_concat([(int(p["mine"][0]), int(p["mine"][1])) for p in parts])
    _, vd = orc.digest_concat([(int(p["mine"][0]), int(p["mine"][2])) for p in parts])
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    assert (n, kd, vd) == (len(want["key"]), orc.digest(want["key"].astype(np.uint64)), orc.digest(want["voff"]))
    sbi = shard.be64([s.first_record_voff] + [int(v) for p in parts for v in p["ent"]] + [len(data) << 16])
    assert sbi == s.splitting_index(g)
