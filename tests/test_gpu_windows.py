"""Bounded-HBM decoding (SURVEY.md 8a a8, a9 and the 60 GB configs C3/C5):
files decoded window by window with the next record's position carried
across windows, split-local opens that read only their byte range, bounded
batches with a resumable cursor, validation stringency, getProgress's
position, and the write-time .splitting-bai -- all against the oracle.
Small windows force many windows on small files, so every path that a 60 GB
file takes runs here in seconds."""
import os
import struct
import zlib

import numpy as np
import pytest

import hbam
import orc
from hbam import synth
from test_gpu_parity import FIELDS, assert_same_records

ALL = (1 << 64) - 1


def recompress(stream, u: bytes) -> bytes:
    """The stream's blocks re-cut from new inflated bytes u (zlib level 5):
    a valid BGZF file carrying whatever records u holds."""
    out = bytearray()
    for b in stream.blocks:
        a, n = int(b["ustart"]), int(b["isize"])
        raw = bytes(u[a:a + n])
        co = zlib.compressobj(5, zlib.DEFLATED, -15)
        c = co.compress(raw) + co.flush()
        total = 18 + len(c) + 8
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", total - 1)
        out += c + struct.pack("<II", zlib.crc32(raw) & 0xFFFFFFFF, n)
    return bytes(out)


def _digest(r):
    kx = np.bitwise_xor.reduce(r["key"].view(np.uint64)) if len(r["key"]) else np.uint64(0)
    return int(kx), int(r["voff"].astype(np.uint64).sum(dtype=np.uint64))


WINDOW_CASES = [
    dict(n_records=20000),                        # short reads
    dict(n_records=12000, block_payload=4096),    # many small blocks, straddling records
    dict(n_records=30, mode="long"),              # records span blocks and windows
    dict(n_records=40, mode="long", all_unmapped=True),  # long Murmur keys
    dict(n_records=6000, level=1, eof_block=False),
    dict(n_records=5000, block_payload=65536, level=6),  # ISIZE 65536
]

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("window", [1 << 16, 150_000])
@pytest.mark.parametrize("kw", WINDOW_CASES, ids=[str(i) for i in range(len(WINDOW_CASES))])
def test_windows_match_oracle(kw, window):
    data, info = synth.make_bam(**kw)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    # a window re-reads the blocks its predecessor could not finish (the
    # record that straddles its end): per pass at most about 3 blocks a
    # window, plus the next window's bytes staged while this one decodes
    # (Pipeline::stage; one window of read-ahead may go unused at the end)
    csize = int(s.blocks["csize"].max())
    per_pass = len(data) * (1 + 3 * csize / window) + 3 * window
    with hbam.BamFile(data, window_bytes=window) as f:
        h = f.header()
        n0 = f.bytes_read()
        got = f.decode_all()
        assert got["status"] == 0 and got["next_voff"] == ALL
        assert_same_records(got, want, s.data)
        assert f.bytes_read() - n0 < per_pass
        for g in (1, 3, 4096):
            n0 = f.bytes_read()
            assert f.splitting_index(g) == s.splitting_index(g)
            assert f.bytes_read() - n0 < per_pass
        n0 = f.bytes_read()
        st = f.decode_span_device(h["first_record_voff"], ALL)
        assert st["status"] == 0 and st["records"] == len(want["key"])
        assert (st["key_xor"], st["voff_sum"]) == _digest(want)
        assert f.bytes_read() - n0 < per_pass
        if len(data) > 4 * window:
            assert st["windows"] >= 3


@pytest.mark.parametrize("window", [1 << 16, 1 << 30])
def test_bounded_batches_resume(window):
    data, _ = synth.make_bam(15000, block_payload=8192)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    with hbam.BamFile(data, window_bytes=window) as f:
        first = f.header()["first_record_voff"]
        for m in (1, 7, 1000, 4096):
            parts = list(f.iter_batches(first, ALL, m))
            assert all(0 < len(p["key"]) <= m for p in parts)
            for name in FIELDS:
                np.testing.assert_array_equal(np.concatenate([p[name] for p in parts]), want[name], err_msg=name)
            # next_voff of a batch is the voff of the following record
            for a, b in zip(parts, parts[1:]):
                assert a["next_voff"] == b["voff"][0]
        # a split inside the file, batches of 333
        vo = want["voff"]
        vs, ve = int(vo[1234]), int(vo[9876])
        rc, wsp = s.decode_span(vs, ve)
        got = np.concatenate([p["key"] for p in f.iter_batches(vs, ve, 333)])
        np.testing.assert_array_equal(got, wsp["key"])


def test_split_local_open_reads_its_range(tmp_path):
    """hbam_open(path) maps the file and copies only the windows a decode
    needs: a split in the middle reads about its own length (plus the window
    that finishes its last record), not the file."""
    data, _ = synth.make_bam(60000)
    path = os.path.join(tmp_path, "c.bam")
    open(path, "wb").write(data)
    size = len(data)
    s = orc.Stream(data)
    window = 256 * 1024
    with hbam.BamFile(path=path, window_bytes=window) as f:
        after_header = f.bytes_read()
        assert after_header <= window
        a, b = size // 3, 2 * size // 3
        (vs, ve), = f.get_splits([a], [b - a])
        after_guess = f.bytes_read()
        assert after_guess - after_header < 512 * 1024
        got = f.decode_span(vs, ve)
        read = f.bytes_read() - after_guess
        assert (b - a) * 0.9 < read < (b - a) + 2 * window
        rc, want = s.decode_span(vs, ve)
        assert_same_records(got, want, s.data)


def test_prefetch_then_device_decode():
    data, _ = synth.make_bam(30000)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    with hbam.BamFile(data, window_bytes=300_000) as f:
        f.prefetch(0, len(data))
        n0 = f.bytes_read()
        st = f.decode_span_device(f.header()["first_record_voff"], ALL, timing=True)
        assert f.bytes_read() == n0  # every window attached to the HBM copy
        assert st["records"] == len(want["key"]) and (st["key_xor"], st["voff_sum"]) == _digest(want)


def _patched(data, rec, offset, fmt, value):
    s = orc.Stream(data, stringency=orc.SILENT)
    rc, r = s.decode_all()
    u = bytearray(s.data)
    struct.pack_into(fmt, u, int(r["offset"][rec]) + offset, value)
    return recompress(s, bytes(u))


# (record, byte offset in the record, struct format, value): each breaks one
# SAMRecord.isValid rule of a record of the 3000-record synthetic BAM
STRICT_CASES = [
    (1700, 14, "<H", 1),              # bin != reg2bin
    (1700, 18, "<H", 0x2),            # unpaired read with the proper-pair flag
    (900, 18, "<H", 0x1 | 0x2 | 0x4 | 0x40 | 0x20),  # unmapped read, MAPQ != 0
    (900, 24, "<i", -1),              # mate reference "*" with a mate position
    (1200, 8, "<i", -1),              # refID set, position "*"
    (2500, 28, "<i", 300000000),      # mate position past the reference
]


@pytest.mark.parametrize("case", STRICT_CASES, ids=[str(i) for i in range(len(STRICT_CASES))])
def test_strict_validation_matches_oracle(case):
    data, _ = synth.make_bam(3000)
    bad = _patched(data, *case)
    for stringency in (hbam.STRICT, hbam.LENIENT, hbam.SILENT):
        s = orc.Stream(bad, stringency=stringency)
        rc, want = s.decode_all()
        assert rc == (1 if stringency == hbam.STRICT else 0)
        for window in (1 << 16, 1 << 30):
            with hbam.BamFile(bad, stringency=stringency, window_bytes=window) as f:
                got = f.decode_all(raise_on_error=False)
                assert got["status"] == rc
                assert_same_records(got, want)


def test_structural_decode_errors_fail_lenient_too():
    data, _ = synth.make_bam(3000)
    s0 = orc.Stream(data, stringency=orc.SILENT)
    rc, r = s0.decode_all()
    lrn = int(r["l_read_name"][1500])
    bad = _patched(data, 1500, 36 + lrn, "<I", (150 << 4) | 9)  # cigar op 9
    for stringency, code in ((hbam.STRICT, 1), (hbam.LENIENT, 1), (hbam.SILENT, 0)):
        rc, want = orc.Stream(bad, stringency=stringency).decode_all()
        assert rc == code
        with hbam.BamFile(bad, stringency=stringency) as f:
            got = f.decode_all(raise_on_error=False)
            assert got["status"] == code
            assert_same_records(got, want)


def _block_end(s, pos):
    for b in s.blocks:
        if int(b["ustart"]) <= pos < int(b["ustart"]) + int(b["isize"]):
            return int(b["coff"]) + int(b["csize"])
    raise AssertionError(pos)


@pytest.mark.parametrize("window", [0, 1 << 16])
def test_reader_position_follows_htsjdk_read_ahead(window):
    """getProgress's in.position(): the end of the block holding the last byte
    of the record after the current one (BAMFileIndexIterator reads one
    ahead), or of the current one at the end of the split -- also when that
    next record lies in the next window (64 KiB windows: batches end at
    window ends)."""
    data, _ = synth.make_bam(4000, block_payload=16384)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    ends = [int(want["offset"][i]) + 36 + int(want["rest_len"][i]) - 1 for i in range(len(want["key"]))]
    vo = want["voff"]
    vs, ve = int(vo[100]), int(vo[3000])
    with hbam.BamFile(data, window_bytes=window) as f:
        done, batches = 0, 0
        for batch in f.iter_batches(vs, ve, 500):
            n = len(batch["key"])
            for i in list(range(0, n, 37)) + [n - 1]:
                k = 100 + done + i
                ahead = k + 1 if k + 1 < 3000 else k
                assert f.reader_position(i) == _block_end(s, ends[ahead]), (done, i)
            done += n
            batches += 1
        assert done == 2900
        if window:
            assert batches > 2900 // 500 + 1  # window ends cut batches short
        # a call of another kind moves the cursor: no position until the next batch
        f.file_stats()
        with pytest.raises(hbam.HbamError) as e:
            f.reader_position(0)
        assert e.value.code == hbam.E_STATE


@pytest.mark.parametrize("window", [0, 1 << 16])
def test_batch_size_changing_mid_split(window):
    """A caller that changes max_records between calls of one split: batches
    that are not blocks of the window's batch-major columns take the
    per-column copies.  Every batch's data holds the rests alone, back to
    back (rest_off[0] = 0, data_len = sum of rest_len), byte-equal to the
    oracle's, and positions still follow the read-ahead rule."""
    data, _ = synth.make_bam(6000, block_payload=16384)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    ends = [int(want["offset"][i]) + 36 + int(want["rest_len"][i]) - 1 for i in range(len(want["key"]))]
    vo = want["voff"]
    lo, hi = 50, 5500
    with hbam.BamFile(data, window_bytes=window) as f:
        v, done, sizes = int(vo[lo]), 0, [700, 333, 700, 1, 1024, 700]
        j = 0
        while v < int(vo[hi]):
            r = f.decode_span(v, int(vo[hi]), max_records=sizes[j % len(sizes)])
            j += 1
            n = len(r["key"])
            assert n and r["status"] == 0
            k0 = lo + done
            np.testing.assert_array_equal(r["key"], want["key"][k0:k0 + n])
            np.testing.assert_array_equal(r["rest_len"], want["rest_len"][k0:k0 + n])
            assert int(r["rest_off"][0]) == 0 and len(r["data"]) == int(r["rest_len"].astype(np.int64).sum())
            for i in range(n):
                off, ln = int(want["offset"][k0 + i]) + 36, int(want["rest_len"][k0 + i])
                assert r["data"][int(r["rest_off"][i]):int(r["rest_off"][i]) + ln] == s.data[off:off + ln], (k0, i)
            for i in sorted({0, n // 2, n - 1}):
                ahead = min(k0 + i + 1, hi - 1)
                assert f.reader_position(i) == _block_end(s, ends[ahead]), (k0, i)
            done += n
            v = r["next_voff"]
        assert done == hi - lo and j > len(sizes)


@pytest.mark.parametrize("g", [1, 2, 10, 4096])
def test_write_time_index_matches_process_alignment(test_bam, g):
    """SplittingBAMIndexer(out, g).processAlignment over every record, then
    finish(size) (SplittingBAMIndexer.java:186-202, 240-243), entries picked
    on the GPU; and TestSplittingBAMIndexer.java:27-32's relation: the same
    SplittingBAMIndex as index() and the same bamSize."""
    s = orc.Stream(test_bam)
    rc, r = s.decode_all()
    v = [int(x) for x in r["voff"]]
    want = [v[i] for i in range(len(v)) if i == 0 or (i + 1) % g == 0] + [len(test_bam) << 16]
    got = hbam.splitting_index_for_records(r["voff"], g, len(test_bam))
    assert got == b"".join(x.to_bytes(8, "big") for x in want)
    idx = s.splitting_index(g)
    as_set = lambda b: {int.from_bytes(b[i:i + 8], "big") for i in range(0, len(b), 8)}
    assert as_set(got) == as_set(idx)


def test_continuation_at_an_empty_block_is_eof():
    """[htsjdk] an empty BGZF block right after an exhausted one reads as EOF:
    a window that starts at such a block ends the span."""
    d1, _ = synth.make_bam(3000, eof_block=True)
    d2, _ = synth.make_bam(3000, seed=99, eof_block=False)
    s2 = orc.Stream(d2)
    # the second file's records after the first's EOF block: unreachable
    h2 = s2.header_end
    blk = s2.blocks
    # the data blocks of file 2 that hold only records (start after its header)
    k = int(np.searchsorted(blk["ustart"], h2, side="right"))
    tail = d2[int(blk["coff"][k]):]
    data = d1 + tail
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0 and len(want["key"]) == 3000
    for window in (1 << 16, 1 << 30):
        with hbam.BamFile(data, window_bytes=window) as f:
            got = f.decode_all()
            assert_same_records(got, want)
            assert f.splitting_index(5) == s.splitting_index(5)


def test_reopened_splits_reuse_cached_blocks(tmp_path):
    """hbam_mem: the device and page-locked blocks a closed split frees are
    handed to the next open in the process with their old contents.  Opening
    different files in turn (short reads, long reads, windowed, batched) must
    give the oracle's records every time -- nothing may rely on fresh memory."""
    files = []
    for n, mode in ((40000, "short"), (300, "long"), (25000, "short")):
        data, _ = synth.make_bam(n, mode=mode, seed=77 + n)
        p = tmp_path / f"r{n}.bam"
        p.write_bytes(data)
        s = orc.Stream(data)
        rc, want = s.decode_all()
        assert rc == 0
        files.append((str(p), want, s.data))
    for rnd in range(2):
        for path, want, u in files:
            for window, batch in ((0, 0), (200_000, 7000)):
                with hbam.BamFile(path=path, window_bytes=window) as f:
                    first = f.header()["first_record_voff"]
                    if batch:
                        parts, v = [], first
                        while v < ALL:
                            r = f.decode_span(v, ALL, max_records=batch)
                            if len(r["key"]) == 0:
                                break
                            parts.append(r)
                            v = r["next_voff"]
                        got = {k: np.concatenate([p_[k] for p_ in parts]) for k in ("key", "voff", "pos", "flag")}
                        for k in got:
                            assert np.array_equal(got[k], want[k]), (rnd, path, window, k)
                    else:
                        got = f.decode_all()
                        assert_same_records(got, want, u)
    # the closed splits left their blocks in the process caches; releasing
    # them empties the caches, and a later open allocates afresh
    assert hbam.release_cached_memory() > 0
    assert hbam.release_cached_memory() == 0
    path, want, u = files[0]
    with hbam.BamFile(path=path) as f:
        assert_same_records(f.decode_all(), want, u)


def _long_cigar_cases():
    """(record, op index, new op, new len) on the 40-record long-read BAM:
    each edit breaks (or keeps) one Cigar.isValid / alignment rule inside a
    cigar of 150-750 operators -- the records k_rec_check validates with a
    whole wave (record_invalid_wave)."""
    return [
        (1, 100, 1, 3), (1, 101, 1, 3),      # I next to I / an I inside a run
        (2, 200, 2, 4), (2, 0, 2, 4),        # D in the middle, D first
        (3, 57, 5, 10), (3, -1, 5, 10),      # H in the middle / last
        (4, 1, 4, 7), (4, 120, 4, 7),        # S second / in the middle
        (6, 30, 6, 2), (6, -1, 6, 2),        # P between real ops / last
        (7, 300, 0, 0), (7, 64, 0, 0),       # zero-length M (chunk boundary)
        (8, 63, 1, 2), (8, 127, 2, 2),       # I / D at chunk ends
        (9, 200, 9, 5),                      # operator 9 (structural: LENIENT too)
        (10, 10, 3, 200000000),              # N run off the reference end
        (11, 250, 0, 151),                   # M length: cigar read length != l_seq
        (13, 70, "X", 0), (14, 140, "=", 0),  # an M relabelled X / = (same length): still valid
    ]


@pytest.mark.parametrize("case", _long_cigar_cases(), ids=[str(i) for i in range(len(_long_cigar_cases()))])
def test_long_cigar_validation_matches_oracle(case):
    rec, k, op, ln = case
    data, _ = synth.make_bam(40, mode="long")
    s0 = orc.Stream(data, stringency=orc.SILENT)
    rc, r = s0.decode_all()
    ncig = int(r["n_cigar"][rec])
    assert ncig > 64
    lrn = int(r["l_read_name"][rec])
    k = k % ncig
    if isinstance(op, str):  # relabel the first M at or after k, keeping its length
        u = s0.data
        at = int(r["offset"][rec]) + 36 + lrn
        while struct.unpack_from("<I", u, at + 4 * k)[0] & 15:
            k += 1
        ln = struct.unpack_from("<I", u, at + 4 * k)[0] >> 4
        op = {"X": 8, "=": 7}[op]
    bad = _patched(data, rec, 36 + lrn + 4 * k, "<I", (ln << 4) | op)
    for stringency in (hbam.STRICT, hbam.LENIENT):
        want_rc, want = orc.Stream(bad, stringency=stringency).decode_all()
        with hbam.BamFile(bad, stringency=stringency) as f:
            got = f.decode_all(raise_on_error=False)
        assert got["status"] == want_rc, (case, stringency)
        assert_same_records(got, want)


@pytest.mark.parametrize("cap", [150_000, 1])
def test_bounded_batches_cap_their_rest_bytes(monkeypatch, cap):
    """A bounded batch hands its rests to Java as one direct ByteBuffer (int
    capacity, int positions: GpuBAMRecordReader.recordAt): the cursor ends a
    batch before its rests pass the cap (2 GiB; HBAM_MAX_BATCH_BYTES lowers
    it here), one record at least, and the batches still cover the split in
    order.  Long reads (10-50 kb) reach a 150 KB cap every few records."""
    data, _ = synth.make_bam(80, mode="long")
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    monkeypatch.setenv("HBAM_MAX_BATCH_BYTES", str(cap))
    with hbam.BamFile(data) as f:
        first = f.header()["first_record_voff"]
        got = list(f.iter_batches(first, ALL, max_records=1 << 20))
    assert len(got) > 4
    for b in got:
        assert b["status"] == 0
        assert len(b["data"]) <= cap or len(b["key"]) == 1
    keys = np.concatenate([b["key"] for b in got])
    voffs = np.concatenate([b["voff"] for b in got])
    np.testing.assert_array_equal(keys, want["key"])
    np.testing.assert_array_equal(voffs, want["voff"])
    u = s.data
    rests = b"".join(u[o + 36:o + 36 + n] for o, n in zip(want["offset"].tolist(), want["rest_len"].tolist()))
    assert b"".join(b["data"] for b in got) == rests
