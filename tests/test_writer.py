"""BAM write path host side: BAMRecordWriter
(BAMRecordWriter.java:51-168) over the GPU-deflated BGZF stream --
hbam.writer.BamWriter, the mirror of java/.../GpuBAMRecordWriter.java.

Checked: the file bytes are the stock stream's (test.bam's payload cut every
HTSJDK_BLOCK_SIZE bytes at level 5, no EOF terminator; the oracle's zlib
recompression, pinned by test_bgzf_write on the reference's fixtures), for
buffers of 1, 3 and 1024 blocks (several GPU calls, or one), and the
write-time .splitting-bai equals the one the reference's read-time indexer
(SplittingBAMIndexer.index, restated by orc.scan) makes of the written file.
The CPU tests run the same host logic with the oracle's compressor standing in
for the GPU call; the GPU tests run the product."""
import io

import pytest

import orc
from conftest import golden_path
from test_bgzf_write import split_bgzf


def _records():
    """(header bytes, record byte strings) of test.bam's inflated payload."""
    u, _, _ = split_bgzf(open(golden_path("test.bam"), "rb").read())
    l_text = int.from_bytes(u[4:8], "little")
    p = 8 + l_text
    n_ref = int.from_bytes(u[p:p + 4], "little")
    p += 4
    for _ in range(n_ref):
        p += 4 + int.from_bytes(u[p:p + 4], "little") + 4
    hdr, recs = u[:p], []
    while p < len(u):
        bs = int.from_bytes(u[p:p + 4], "little")
        recs.append(u[p:p + 4 + bs])
        p += 4 + bs
    assert p == len(u) and len(recs) == 2277
    return u, hdr, recs


def _write(buffer_blocks, granularity):
    from hbam.writer import BamWriter
    u, hdr, recs = _records()
    out, sbi = io.BytesIO(), io.BytesIO()
    w = BamWriter(out, header=hdr, buffer_blocks=buffer_blocks, splitting_bai=sbi, granularity=granularity)
    for r in recs:
        w.write_record(r)
    w.close()
    return u, out.getvalue(), sbi.getvalue()


def _check(u, got, sbi, granularity):
    import hbam
    bs = hbam.HTSJDK_BLOCK_SIZE
    lens = [min(bs, len(u) - p) for p in range(0, len(u), bs)]
    assert got == orc.bgzf_compress(u, lens, level=5, eof=False)
    _, want = orc.scan(got, mode="index", granularity=granularity)
    assert sbi == want
    assert len(sbi) == 8 * (1 + (2277 - 1) // granularity + 1 + (2277 % granularity == 0))


@pytest.mark.parametrize("buffer_blocks,granularity", [(1, 100), (3, 7), (1024, 4096)])
def test_writer_host_logic(monkeypatch, buffer_blocks, granularity):
    import hbam.writer as W
    monkeypatch.setattr(W, "bgzf_compress",
                        lambda d, block_lens, level, eof, device: orc.bgzf_compress(d, block_lens, level=level, eof=eof))
    _check(*_write(buffer_blocks, granularity), granularity)


def test_writer_index_records_at_block_starts(monkeypatch):
    """A record that starts exactly where a block starts gets that block's
    address with offset 0 (the stock stream deflates a full buffer at once,
    so getFilePointer() already points past it)."""
    import hbam.writer as W
    monkeypatch.setattr(W, "bgzf_compress",
                        lambda d, block_lens, level, eof, device: orc.bgzf_compress(d, block_lens, level=level, eof=eof))
    out, sbi = io.BytesIO(), io.BytesIO()
    rec = (96).to_bytes(4, "little") + bytes(96)  # 100-byte records: 10 per 1000-byte block
    w = W.BamWriter(out, buffer_blocks=2, splitting_bai=sbi, granularity=1, block=1000)
    for _ in range(45):
        w.write_record(rec)
    w.close()
    z = out.getvalue()
    starts, p = [], 0
    while p < len(z):
        starts.append(p)
        p += int.from_bytes(z[p + 16:p + 18], "little") + 1
    v = [int.from_bytes(sbi.getvalue()[8 * i:8 * i + 8], "big") for i in range(len(sbi.getvalue()) // 8)]
    assert v[:-1] == [starts[i // 10] << 16 | (i % 10) * 100 for i in range(45)]
    assert v[-1] == len(z) << 16


@pytest.mark.gpu
@pytest.mark.parametrize("buffer_blocks,granularity", [(1, 100), (3, 7), (1024, 4096)])
def test_gpu_writer_matches_stock_stream_and_index(buffer_blocks, granularity):
    _check(*_write(buffer_blocks, granularity), granularity)
