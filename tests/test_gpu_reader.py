"""Reading through a Hadoop FileSystem stream (hbam_open_reader) and through
pread of a path, against the oracle.

The reference reads every split through WrapSeekable.openPath(fs, path) over
an FSDataInputStream (util/WrapSeekable.java:56-87; BAMRecordReader.java:147,
BAMInputFormat.java:476) and indexes a plain InputStream front to back
(SplittingBAMIndexer.index(InputStream, ...), :248-290).  Here a Python
positioned-read callback stands in for the JNI glue's FSDataInputStream
reader: splits decode through it (no mmap, no path), the indexer reads a
forward-only stream, and a file shorter than its stated length -- or a local
file truncated while open -- fails with HBAM_E_TRUNC (FileTruncatedException)
instead of a signal."""
import os
import threading

import numpy as np
import pytest

import hbam
import orc
from hbam import synth
from test_gpu_parity import assert_same_records

pytestmark = pytest.mark.gpu
ALL = (1 << 64) - 1


class Reader:
    """PositionedReadable over bytes, recording every call; forward=True
    fails a read behind the last one (an InputStream)."""

    def __init__(self, data, forward=False, fail_at=None, short_at=None):
        self.data = data
        self.forward = forward
        self.fail_at = fail_at      # an offset whose read raises (IOException)
        self.short_at = short_at    # the file really ends here (truncated)
        self.calls = []
        self.pos = 0
        self.busy = threading.Lock()
        self.overlap = False

    def __call__(self, off, n):
        if not self.busy.acquire(blocking=False):
            self.overlap = True  # two calls at once for one ctx
            self.busy.acquire()
        try:
            self.calls.append((off, n))
            if self.forward:
                if off < self.pos:
                    raise IOError(f"backward read at {off} of a stream at {self.pos}")
                self.pos = off + n
            if self.fail_at is not None and off <= self.fail_at < off + n:
                raise IOError("injected read error")
            end = len(self.data) if self.short_at is None else self.short_at
            return bytes(self.data[off:min(off + n, end)])
        finally:
            self.busy.release()


def _splits(f, size, n):
    step = -(-size // n)
    begs = [min(size, k * step) for k in range(n)]
    ends = [min(size, (k + 1) * step) for k in range(n)]
    plan = f.get_splits(begs, [e - b for b, e in zip(begs, ends)])
    return plan


@pytest.mark.parametrize("window", [1 << 16, 0])
def test_splits_through_a_reader_match_the_oracle(window):
    data, _ = synth.make_bam(30000, block_payload=16384)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    r = Reader(data)
    with hbam.BamFile(reader=r, size=len(data), window_bytes=window) as f:
        assert f.header()["first_record_voff"] == s.first_record_voff
        plan = _splits(f, len(data), 5)
        parts = [f.decode_span(vs, ve) for vs, ve in plan]
    got = {k: np.concatenate([p[k] for p in parts]) for k in ("voff", "key")}
    for p in parts:
        assert p["status"] == 0
    # the splits cover every record once, in file order
    assert np.array_equal(got["voff"], want["voff"])
    assert np.array_equal(got["key"], want["key"])
    assert not r.overlap
    assert r.calls and all(off + n <= len(data) for off, n in r.calls)


def test_reader_decode_equals_path_decode(tmp_path):
    data, _ = synth.make_bam(8000, mode="short")
    p = tmp_path / "x.bam"
    p.write_bytes(data)
    with hbam.BamFile(path=str(p), window_bytes=1 << 17) as a, \
            hbam.BamFile(reader=Reader(data), size=len(data), window_bytes=1 << 17) as b:
        ga, gb = a.decode_all(), b.decode_all()
        assert ga["status"] == gb["status"] == 0
        s = orc.Stream(data)
        assert_same_records(gb, s.decode_all()[1], s.data)
        for k in ("key", "voff", "rest_len", "flag"):
            assert np.array_equal(ga[k], gb[k]), k
        for g in (1, 10, 4096):
            assert a.splitting_index(g) == b.splitting_index(g) == s.splitting_index(g)


@pytest.mark.parametrize("g", [1, 2, 10, 4096])
def test_stream_index_reads_front_to_back(test_bam, g):
    """SplittingBAMIndexer.index(InputStream, ...) over a forward-only stream:
    byte-identical to the oracle, every read at or after the last."""
    s = orc.Stream(test_bam)
    r = Reader(test_bam, forward=True)
    with hbam.BamFile(reader=r, size=len(test_bam)) as f:
        assert f.splitting_index(g) == s.splitting_index(g)
    offs = [o for o, _ in r.calls]
    assert offs == sorted(offs)


@pytest.mark.parametrize("g", [1, 2, 10, 4096])
def test_stream_index_many_windows(g):
    data, _ = synth.make_bam(20000, block_payload=8192)
    s = orc.Stream(data)
    r = Reader(data, forward=True)
    with hbam.BamFile(reader=r, size=len(data), window_bytes=150_000) as f:
        assert f.splitting_index(g) == s.splitting_index(g)
    offs = [o for o, _ in r.calls]
    assert offs == sorted(offs)
    # each byte crosses once (a window keeps its predecessor's tail on the device)
    assert sum(n for _, n in r.calls) <= len(data) + (1 << 20)


def test_truncated_stream_is_file_truncated():
    data, _ = synth.make_bam(20000, block_payload=16384)
    r = Reader(data, short_at=len(data) // 2)
    with hbam.BamFile(reader=r, size=len(data), window_bytes=1 << 18) as f:
        with pytest.raises(hbam.HbamError) as e:
            f.decode_all()
        assert e.value.code == hbam.E_TRUNC
        assert "truncated" in str(e.value)


def test_reader_error_is_io_error():
    data, _ = synth.make_bam(20000, block_payload=16384)
    r = Reader(data, fail_at=len(data) // 2)
    with hbam.BamFile(reader=r, size=len(data), window_bytes=1 << 18) as f:
        with pytest.raises(hbam.HbamError) as e:
            f.decode_all()
        assert e.value.code == hbam.E_IO


def test_truncated_header_fails_open():
    data, _ = synth.make_bam(200)
    with pytest.raises(hbam.HbamError) as e:
        hbam.BamFile(reader=Reader(data, short_at=10), size=len(data))
    assert e.value.code in (hbam.E_TRUNC, hbam.E_IO, hbam.E_FORMAT)


def test_local_file_truncated_while_open(tmp_path):
    """hbam_open checks the file's length before each read of its mapping: a
    file cut short under an open ctx is a FileTruncatedException on the call
    that reads there (the copy from the mapping raised SIGBUS before)."""
    data, _ = synth.make_bam(20000, block_payload=16384)
    p = tmp_path / "t.bam"
    p.write_bytes(data)
    with hbam.BamFile(path=str(p), window_bytes=1 << 18) as f:
        first = f.header()["first_record_voff"]
        os.truncate(p, len(data) // 3)
        with pytest.raises(hbam.HbamError) as e:
            f.decode_span(first, ALL)
        assert e.value.code == hbam.E_TRUNC


def test_prefetch_through_a_reader():
    data, _ = synth.make_bam(10000)
    r = Reader(data)
    s = orc.Stream(data)
    with hbam.BamFile(reader=r, size=len(data)) as f:
        f.prefetch(0, len(data))
        n = len(r.calls)
        st = f.decode_span_device(f.header()["first_record_voff"], ALL)
        assert st["records"] == len(s.decode_all()[1]["key"])
        assert len(r.calls) == n  # decoded from HBM, no more reads


def test_parallel_reads_match_the_oracle():
    """parallel_reads: the copy threads call the reader at once (disjoint
    ranges, as HDFS positioned reads allow); same records."""
    data, _ = synth.make_bam(60000, block_payload=65280)
    s = orc.Stream(data)
    r = Reader(data)
    with hbam.BamFile(reader=r, size=len(data), parallel_reads=True) as f:
        got = f.decode_all()
    assert got["status"] == 0
    assert_same_records(got, s.decode_all()[1], s.data)
    # the ranges read cover the file, none twice
    spans = sorted(r.calls)
    assert all(a + n <= b for (a, n), (b, _) in zip(spans, spans[1:]))
