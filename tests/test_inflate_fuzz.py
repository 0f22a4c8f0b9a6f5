"""GPU inflate vs zlib (the oracle) on corrupted BGZF blocks.

The all-lane speculative Huffman decoder must reproduce zlib's inflate()
exactly as [htsjdk] BlockGunzipper drives it (one call, ISIZE bytes of output
space, CRC off): same status (OK / DataFormatException -> E_IO / "Did not
inflate expected amount" -> E_FORMAT) and, on success, the same bytes.  The
corruptions hit the paths plain data never reaches: invalid codes, distances
too far back, input exhausted mid-symbol, and ISIZE footers smaller or larger
than the real output (zlib's post-full lookahead decides those)."""
import struct

import numpy as np
import pytest

import hbam
import orc
from hbam import synth

pytestmark = pytest.mark.gpu

VARIANTS = [
    dict(level=5),
    dict(level=1),
    dict(level=9),
    dict(level=0),
    dict(strategy="fixed"),
    dict(strategy="huffman"),
    dict(strategy="rle"),
]


def _status_and_bytes_hbam(data):
    try:
        with hbam.BamFile(data, bam=False) as f:
            n = int(sum(int(x) for x in f.blocks()["isize"]))
            return hbam.OK, f.read_inflated(0, n)
    except hbam.HbamError as e:
        return e.code, None


def _status_and_bytes_oracle(data):
    try:
        s = orc.Stream(data, check_crc=False, parse_header=False)
        return hbam.OK, s.data
    except orc.OracleError as e:
        return e.code, None


def _corruptions(d, rng, n):
    s = orc.Stream(d, parse_header=False)
    blocks = [b for b in s.blocks if int(b["isize"]) > 0]
    for _ in range(n):
        b = blocks[int(rng.integers(len(blocks)))]
        coff, csize, isize = int(b["coff"]), int(b["csize"]), int(b["isize"])
        out = bytearray(d)
        mode = int(rng.integers(4))
        if mode == 0:  # one byte anywhere in CDATA
            at = coff + 18 + int(rng.integers(csize - 26))
            out[at] ^= int(rng.integers(1, 256))
        elif mode == 1:  # the last CDATA bytes (end-of-block region)
            at = coff + csize - 8 - 1 - int(rng.integers(min(4, csize - 26)))
            out[at] ^= int(rng.integers(1, 256))
        elif mode == 2:  # ISIZE smaller than the real output
            struct.pack_into("<I", out, coff + csize - 4, int(rng.integers(0, isize)))
        else:  # ISIZE larger
            struct.pack_into("<I", out, coff + csize - 4, min(65536, isize + 1 + int(rng.integers(64))))
        yield bytes(out)


@pytest.mark.parametrize("kw", VARIANTS, ids=[str(i) for i in range(len(VARIANTS))])
def test_corrupted_blocks_match_zlib(kw):
    d, _ = synth.make_bam(300, block_payload=8192, **kw)
    rng = np.random.default_rng(11 + len(str(kw)))
    seen = set()
    for bad in _corruptions(d, rng, 40):
        want_rc, want = _status_and_bytes_oracle(bad)
        got_rc, got = _status_and_bytes_hbam(bad)
        seen.add(want_rc)
        assert got_rc == want_rc
        if want_rc == hbam.OK:
            assert got == want
    assert len(seen) >= 2  # the corruptions reached more than one outcome


def test_isize_exactly_short_by_one_symbol():
    """ISIZE = real size - 1 on every block: zlib fills the buffer and peeks the
    next symbol (no error); the stream is the real output minus one byte per block."""
    d, _ = synth.make_bam(300, block_payload=8192)
    s = orc.Stream(d, parse_header=False)
    out = bytearray(d)
    for b in s.blocks:
        coff, csize, isize = int(b["coff"]), int(b["csize"]), int(b["isize"])
        if isize:
            struct.pack_into("<I", out, coff + csize - 4, isize - 1)
    bad = bytes(out)
    want_rc, want = _status_and_bytes_oracle(bad)
    got_rc, got = _status_and_bytes_hbam(bad)
    assert got_rc == want_rc == hbam.OK
    assert got == want


def _fixed_block_with_distance_code(dcode, nlit=400):
    """One BGZF block: a fixed-Huffman DEFLATE block of nlit literals, a
    length-3 match with distance code dcode (30 and 31 are invalid in
    DEFLATE), nlit more literals and the end-of-block code.  The match lies
    thousands of bits before the end, in the decoder's fast region."""
    import zlib
    bits, nbits = 0, 0

    def put(v, n):  # n bits, LSB first
        nonlocal bits, nbits
        bits |= v << nbits
        nbits += n

    def put_code(c, n):  # a Huffman code, MSB first
        put(int(format(c, "0%db" % n)[::-1], 2), n)

    def lit(v):
        if v < 144:
            put_code(0x30 + v, 8)
        else:
            put_code(0x190 + v - 144, 9)

    rng = np.random.default_rng(dcode)
    body = bytes(rng.integers(65, 91, nlit, dtype=np.uint8))
    put(1, 1)  # BFINAL
    put(1, 2)  # fixed Huffman
    for b in body:
        lit(b)
    put_code(1, 7)  # length code 257: length 3
    put_code(dcode, 5)  # distance code, 5 bits (no extra bits for 0-3; 30/31 invalid)
    if dcode >= 4:
        put(0, (dcode - 2) // 2)
    for b in body:
        lit(b)
    put_code(0, 7)  # end of block
    cdata = bits.to_bytes((nbits + 7) // 8, "little")
    out = body + (body[-4:-1] if dcode == 3 else b"...") + body  # (only the length matters for ISIZE)
    isize = len(out)
    hdr = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", len(cdata) + 25)
    blk = hdr + cdata + struct.pack("<II", zlib.crc32(out) & 0xffffffff, isize)
    eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return blk + eof


@pytest.mark.parametrize("dcode", [30, 31])
def test_invalid_distance_code_in_fast_region(dcode):
    """zlib rejects distance codes 30 and 31 ("invalid distance code" ->
    E_IO); the GPU decoder must too, also when the code is decoded by the
    branch-free fast path (the kind of a K_BAD distance entry has bit 0
    clear, which the fast path's test once missed)."""
    data = _fixed_block_with_distance_code(dcode)
    want_rc, _ = _status_and_bytes_oracle(data)
    got_rc, _ = _status_and_bytes_hbam(data)
    assert want_rc == hbam.E_IO
    assert got_rc == want_rc


def test_valid_distance_code_fixture_decodes():
    """The same construction with a valid distance code decodes to zlib's bytes."""
    data = _fixed_block_with_distance_code(3)
    want_rc, want = _status_and_bytes_oracle(data)
    got_rc, got = _status_and_bytes_hbam(data)
    assert want_rc == got_rc
    assert got == want
