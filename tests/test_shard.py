"""Multi-process sharded read (hbam.shard) on CPU with gloo.

Each rank stands in the oracle as its shard decoder (test infrastructure), so
these tests pin the host logic of the multi-GPU path: byte splits, the
BAMSplitGuesser-based virtual splits, the empty-split merge of
BAMInputFormat.java:497-513, global ordinals and the gathered .splitting-bai.
The GPU decoder behind the same logic is covered by test_gpu_shard.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import orc
from hbam import shard, synth


GUESS_BYTES = 3 * 0xFFFF + 0xFFFE  # BAMSplitGuesser MAX_BYTES_READ (BAMSplitGuesser.java:66-73)


class OracleDecoder:
    """The oracle as a rank's decoder, with the byte accounting of a split
    reader: BAMSplitGuesser reads at most GUESS_BYTES from the split start,
    and BAMRecordReader reads from its first block to the end of the block
    holding its last record's last byte (WrapSeekable seeks, no more)."""

    def __init__(self, data):
        self.s = orc.Stream(data)
        self.read = 0

    def guess_record_starts(self, begs, ends):
        self.read += sum(min(e - b, GUESS_BYTES) for b, e in zip(begs, ends))
        return [self.s.guess_record_start(b, e) for b, e in zip(begs, ends)]

    def decode_span(self, vs, ve):
        rc, r = self.s.decode_span(vs, ve)
        assert rc == 0
        if len(r["voff"]):
            last = int(r["offset"][-1]) + 36 + int(r["rest_len"][-1]) - 1
            bl = self.s.blocks
            k = int(np.searchsorted(bl["ustart"] + bl["isize"], last, side="right"))
            self.read += int(bl["coff"][k]) + int(bl["csize"][k]) - (vs >> 16)
        return r

    def bytes_read(self):
        return self.read


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


WINDOW = 256 * 1024  # GPU decoder: compressed bytes per HBM window


def _worker(rank, world, port, path, outdir, granularity, use_gpu):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if use_gpu:
        import hbam  # split-local: the rank maps the file and copies only the windows it decodes
        dec = hbam.BamFile(path=path, device=0, window_bytes=WINDOW)
        first = dec.header()["first_record_voff"]
    else:
        dec = OracleDecoder(open(path, "rb").read())
        first = dec.s.first_record_voff

    def all_gather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    rd = shard.ShardedBamReader(dec, os.path.getsize(path), first, rank, world, all_gather)
    recs, base, total, sbi = rd.run(granularity)
    keys = recs["key"] if recs is not None else np.zeros(0, np.int64)
    voffs = recs["voff"] if recs is not None else np.zeros(0, np.uint64)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), key=keys, voff=voffs, base=base, total=total,
             sbi=np.frombuffer(sbi, np.uint8) if sbi is not None else np.zeros(0, np.uint8),
             bytes_read=dec.bytes_read())
    dist.destroy_process_group()


def run_sharded(data, world, granularity, tmp_path, use_gpu=False):
    path = os.path.join(tmp_path, "in.bam")
    open(path, "wb").write(data)
    mp.spawn(_worker, args=(world, _free_port(), path, str(tmp_path), granularity, use_gpu), nprocs=world,
             join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    return parts


def check_against_oracle(data, parts, granularity):
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    keys = np.concatenate([p["key"] for p in parts])
    voffs = np.concatenate([p["voff"] for p in parts])
    np.testing.assert_array_equal(voffs, want["voff"])
    np.testing.assert_array_equal(keys, want["key"])
    bases = [int(p["base"]) for p in parts]
    assert bases == [int(sum(len(q["voff"]) for q in parts[:r])) for r in range(len(parts))]
    assert all(int(p["total"]) == len(want["voff"]) for p in parts)
    assert parts[0]["sbi"].tobytes() == s.splitting_index(granularity)


def check_rank_local_reads(data, parts, slack):
    """Every rank reads about its own FileSplit: its split's bytes plus the
    guesser's window and the tail that finishes its last record (`slack`),
    never the whole file."""
    world = len(parts)
    for r, (a, n) in enumerate(shard.file_splits(len(data), world)):
        got = int(parts[r]["bytes_read"])
        assert got <= n + slack, (r, got, n, slack)
    assert sum(int(p["bytes_read"]) for p in parts) <= len(data) + world * slack


def test_file_splits_cover_the_file():
    for size, world in ((10, 3), (1000, 8), (7, 8)):
        sp = shard.file_splits(size, world)
        assert len(sp) == world
        assert sp[0][0] == 0 and sum(n for _, n in sp) == size
        for (a, n), (b, _) in zip(sp, sp[1:]):
            assert a + n == b


def test_merge_empty_splits_follows_reference():
    # BAMInputFormat.java:497-513: an empty split extends the previous one
    got = shard.merge_empty_splits([(5, 10, False), (20, 30, True), (25, 40, True), (50, 60, False)])
    assert got == [(5, 40), None, None, (50, 60)]
    with pytest.raises(IOError):
        shard.merge_empty_splits([(0, 10, True), (20, 30, False)])


@pytest.mark.parametrize("world,g,kw", [
    (2, 4096, dict(n_records=6000)),
    (3, 7, dict(n_records=4000, block_payload=4096)),          # many straddling records
    (4, 1, dict(n_records=1500, block_payload=8192, level=1)),
    (2, 5, dict(n_records=12, mode="long")),                     # records spanning many blocks
    (8, 4096, dict(n_records=24000)),                            # the 8-GPU node's rank count
    (8, 3, dict(n_records=3000, block_payload=4096)),            # 8 ranks, straddles at every split
])
def test_sharded_read_matches_whole_file(tmp_path, world, g, kw):
    data, _ = synth.make_bam(**kw)
    parts = run_sharded(data, world, g, tmp_path)
    check_against_oracle(data, parts, g)
    check_rank_local_reads(data, parts, GUESS_BYTES + 4 * 65536 + (800_000 if kw.get("mode") == "long" else 0))
