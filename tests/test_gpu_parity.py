"""GPU parity: libhbam (gfx950 kernels, through the C ABI) vs the oracle and
the committed golden vectors.  Bit-exact everywhere (integer/byte work)."""
import hashlib
import zlib

import numpy as np
import pytest

import hbam
import orc
from conftest import golden_path
from hbam import synth

pytestmark = pytest.mark.gpu
ALL = (1 << 64) - 1

FIELDS = ["ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen", "l_read_name", "mapq", "bin",
          "n_cigar", "flag", "key", "voff", "rest_len"]


def assert_same_records(got, want, stream_data=None, p0=None):
    n = len(want["key"])
    assert len(got["key"]) == n
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)
    if stream_data is not None and n:
        # rest bytes (getVariableBinaryRepresentation) byte-exact
        for i in range(0, n, max(1, n // 200)):
            off = int(want["offset"][i]) + 36
            ln = int(want["rest_len"][i])
            a = got["data"][int(got["rest_off"][i]):int(got["rest_off"][i]) + ln]
            assert a == stream_data[off:off + ln], i


def test_test_bam_decode_golden(test_bam, golden):
    g = np.load(golden_path("test.bam.records.npz"))
    with hbam.BamFile(test_bam) as f:
        h = f.header()
        assert h["first_record_voff"] == 0x196A and h["n_ref"] == 84 and f.file_stats()[0] == 13
        assert f.ref(0) == ("1", 249250621)
        r = f.decode_all()
        assert r["status"] == 0
        want = {k: g[k] for k in g.files}
        s = orc.Stream(test_bam)
        assert_same_records(r, want, s.data)
        assert hashlib.sha256(r["key"].tobytes()).hexdigest().startswith("9cec72cb")


def test_test_bam_inflate_bytes(test_bam, golden):
    with hbam.BamFile(test_bam) as f:
        b = f.blocks()
        assert [[int(b["coff"][i]), int(b["csize"][i]), int(b["isize"][i]), int(b["ustart"][i])]
                for i in range(len(b["coff"]))] == golden["blocks"]
        data = f.read_inflated(0, golden["inflated_len"])
        assert hashlib.sha256(data).hexdigest() == golden["inflated_sha256"]


@pytest.mark.parametrize("g", [1, 2, 10, 4096])
def test_test_bam_splitting_index(test_bam, g):
    want = open(golden_path(f"test.bam.g{g}.splitting-bai"), "rb").read()
    with hbam.BamFile(test_bam) as f:
        assert f.splitting_index(g) == want


def test_bgzf_text_fixtures_inflate(golden):
    for name, t in golden["bgzf_text"].items():
        data = open(golden_path(name), "rb").read()
        with hbam.BamFile(data, bam=False) as f:
            b = f.blocks()
            assert [int(x) for x in b["coff"]] == t["coffs"]
            out = f.read_inflated(0, t["len"])
            assert hashlib.sha256(out).hexdigest() == t["sha256"], name


def test_spans_vs_oracle(test_bam):
    s = orc.Stream(test_bam)
    rc, allr = s.decode_all()
    vo = [int(v) for v in allr["voff"]]
    with hbam.BamFile(test_bam) as f:
        rng = np.random.default_rng(3)
        for _ in range(25):
            a, b = sorted(rng.integers(0, len(vo), 2))
            vs, ve = vo[a], (vo[b] if b > a else (1 << 64) - 1)
            rc, want = s.decode_span(vs, ve)
            got = f.decode_span(vs, ve)
            assert_same_records(got, want)
        # split ends expressed as byte offsets | 0xffff (BAMInputFormat.java:495)
        for end in (20000, 65536, 100000, 150000):
            ve = (end << 16) | 0xFFFF
            rc, want = s.decode_span(vo[0], ve)
            assert_same_records(f.decode_span(vo[0], ve), want)


def test_guesser_golden(test_bam, golden):
    begs = [x[0] for x in golden["guesses"]]
    ends = [x[1] for x in golden["guesses"]]
    want = [x[2] for x in golden["guesses"]]
    with hbam.BamFile(test_bam) as f:
        assert f.guess_record_starts(begs, ends) == want


def test_split_planning_golden(test_bam, golden):
    with hbam.BamFile(test_bam) as f:
        sbi = f.splitting_index(4096)
        for p in golden["plans"]:
            assert [list(x) for x in f.get_splits(p["starts"], p["lengths"], sbi)] == p["indexed"]
            assert [list(x) for x in f.get_splits(p["starts"], p["lengths"], None)] == p["probabilistic"]


SYNTH = [
    dict(n_records=3000),
    dict(n_records=3000, level=1),
    dict(n_records=3000, level=9),
    dict(n_records=1200, level=0),                      # stored blocks
    dict(n_records=2500, strategy="fixed"),             # fixed Huffman
    dict(n_records=2500, strategy="huffman"),           # literals only
    dict(n_records=2500, strategy="rle"),               # distance-1 matches
    dict(n_records=2500, strategy="filtered"),
    dict(n_records=800, all_unmapped=True, block_payload=65498, eof_block=False),  # test.bam-like
    dict(n_records=40, mode="long"),                    # records span many blocks
    dict(n_records=60, mode="long", all_unmapped=True),  # every key through k_long_hash
    dict(n_records=2000, block_payload=4096),           # small blocks, many straddles
    dict(n_records=500, block_payload=65536 - 1024, level=6),
    dict(n_records=3000, block_payload=65536, level=6),  # ISIZE 65536: phase-B round path
    dict(n_records=3000, block_payload=65280, level=1),  # ISIZE at the map limit
    dict(n_records=20000, mode="wgs"),                   # C3's binned-quality model
]


@pytest.mark.parametrize("kw", SYNTH, ids=[str(i) for i in range(len(SYNTH))])
def test_synthetic_vs_oracle(kw):
    d, info = synth.make_bam(**kw)
    s = orc.Stream(d)
    rc, want = s.decode_all()
    assert rc == 0
    with hbam.BamFile(d) as f:
        assert f.file_stats() == (info["blocks"], len(s.data))
        got = f.decode_all()
        assert_same_records(got, want, s.data)
        for g in (1, 3, 4096):
            assert f.splitting_index(g) == s.splitting_index(g)
        u = f.read_inflated(0, len(s.data))
        assert u == s.data


def test_header_only_bam():
    d, info = synth.make_bam(0)
    s = orc.Stream(d)
    with hbam.BamFile(d) as f:
        r = f.decode_all()
        assert len(r["key"]) == 0
        assert f.splitting_index(4096) == s.splitting_index(4096)


def _corrupt(d, at, val):
    b = bytearray(d)
    b[at] = val
    return bytes(b)


def test_error_truncated_file():
    d, _ = synth.make_bam(2000)
    cut = d[:len(d) // 2]
    with pytest.raises(hbam.HbamError) as e:
        hbam.BamFile(cut)
    with pytest.raises(orc.OracleError) as e2:
        orc.Stream(cut)
    assert e.value.code == e2.value.code == hbam.E_TRUNC


def test_error_bad_deflate():
    d, _ = synth.make_bam(2000)
    s = orc.Stream(d)
    b1 = s.blocks[1]
    bad = _corrupt(d, int(b1["coff"]) + 18, 0xFF)  # first DEFLATE header byte: type 3 (invalid)
    with pytest.raises(hbam.HbamError) as e:   # surfaces at open or at decode, as in htsjdk
        with hbam.BamFile(bad) as f:
            f.decode_all()
    with pytest.raises(orc.OracleError) as e2:
        orc.Stream(bad)
    assert e.value.code == e2.value.code == hbam.E_IO


def _rewrite_record(d, rec_index, offset, value4):
    """Change 4 bytes of one record and re-compress (valid BGZF, invalid BAM)."""
    import struct
    import zlib
    s = orc.Stream(d)
    rc, r = s.decode_all()
    u = bytearray(s.data)
    p = int(r["offset"][rec_index]) + offset
    u[p:p + 4] = struct.pack("<i", value4)
    out = bytearray()
    for b in s.blocks:
        a, n = int(b["ustart"]), int(b["isize"])
        raw = bytes(u[a:a + n])
        co = zlib.compressobj(5, zlib.DEFLATED, -15)
        c = co.compress(raw) + co.flush()
        total = 18 + len(c) + 8
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", total - 1)
        out += c + struct.pack("<II", zlib.crc32(raw) & 0xFFFFFFFF, n)
    return bytes(out)


@pytest.mark.parametrize("rec,off,val,code", [(700, 0, 20, 1), (700, 4, 999, 3), (1500, 24, -7, 3)])
def test_record_errors_match_oracle(rec, off, val, code):
    d, _ = synth.make_bam(2000)
    bad = _rewrite_record(d, rec, off, val)
    s = orc.Stream(bad)
    rc, want = s.decode_all()
    assert rc == code
    with hbam.BamFile(bad) as f:
        got = f.decode_all(raise_on_error=False)
        assert got["status"] == code
        assert_same_records(got, want)


def test_c2_full_size_vs_oracle():
    """BASELINE config C2 at full size (10 M records, 1.41 GB BGZF): every key
    and voff of the device pipeline, the .splitting-bai (g = 4096) through
    the SplittingBAMIndexer entry point, and through the reader entry point
    (hbam_decode_span in 2 M-record batches) all 11 fixed-field columns, the
    rest lengths and every rest byte (CRC-32 of all rests in record order),
    bit-exact against the oracle."""
    data, info = synth.make_bam(10_000_000, as_numpy=True)
    raw = data.tobytes()
    g = hbam.Gpu(0)
    g.load(data)
    st = g.run()
    assert st["status"] == 0 and st["records"] == 10_000_000
    keys, voffs = g.fetch(st["records"])
    g.close()
    s = orc.Stream(raw)
    rc, want = s.decode_all()
    assert rc == 0
    np.testing.assert_array_equal(voffs, want["voff"])
    np.testing.assert_array_equal(keys, want["key"])
    want_sbi = s.splitting_index(4096)
    # the oracle's rests: the inflated records without their 36-byte heads
    # (records are back to back from the first one to the last one's end)
    u = s.data_array()
    off = want["offset"].astype(np.int64)
    lo, hi = int(off[0]), int(off[-1]) + 36 + int(want["rest_len"][-1])
    head = np.zeros(hi - lo, bool)
    for j in range(36):
        head[off - lo + j] = True
    want_crc = zlib.crc32(u[lo:hi][~head])
    del head, u, s
    with hbam.BamFile(raw, batch_records=1 << 21) as f:
        assert f.splitting_index(4096) == want_sbi
        parts, crc = {k: [] for k in FIELDS}, 0
        for b in f.iter_batches(f.header()["first_record_voff"], ALL, 1 << 21):
            assert b["status"] == 0
            for k in FIELDS:
                parts[k].append(b[k])
            crc = zlib.crc32(b["data"], crc)
    for k in FIELDS:
        np.testing.assert_array_equal(np.concatenate(parts[k]), want[k], err_msg=k)
    assert crc == want_crc


def test_c4_long_reads_vs_oracle():
    """C4-like ONT reads (10-50 kb, records spanning several BGZF blocks, heavy
    aux tags, 10 % unmapped -> Murmur over ~100 KB rests)."""
    data, info = synth.make_bam(600, mode="long", seed=0x48424D04)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0
    with hbam.BamFile(data) as f:
        got = f.decode_all()
        assert_same_records(got, want, s.data)
        for gran in (1, 5, 4096):
            assert f.splitting_index(gran) == s.splitting_index(gran)


def test_inflate_token_count_is_consistent():
    """hbam_inflate_token_count (the bench's phase-A traffic denominator):
    the LZ77 tokens of the last pass lie between U / 258 (every token a
    longest match) and U (every token one literal), and a second pass over the
    same span writes the same number."""
    d, _ = synth.make_bam(20000)
    s = orc.Stream(d)
    u = len(s.data)
    with hbam.BamFile(d) as f:
        first = f.header()["first_record_voff"]
        st = f.decode_span_device(first, (1 << 64) - 1)
        t1 = f.inflate_token_count()
        assert st["records"] == 20000
        assert u // 258 <= t1 <= u, (t1, u)
        f.decode_span_device(first, (1 << 64) - 1)
        assert f.inflate_token_count() == t1
