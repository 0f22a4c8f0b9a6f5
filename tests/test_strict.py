"""Validation stringency (hadoopbam.samheaderreader.validation-stringency,
util/SAMHeaderReader.java:45-46; BAMRecordReader.java:142,192-194).

CPU: the two restatements of htsjdk's SAMRecord.isValid rule list (C oracle
orc_record_invalid, Python py_oracle.record_invalid) agree on mutated records,
and test.bam -- which the reference reads under htsjdk's default STRICT in
TestSplittingBAMIndexer.java:27-32 -- passes every rule.  Parity with htsjdk
itself is unpinned beyond that (no JVM here; no reference test asserts a
validation error).  The GPU rules are compared with the oracle in
test_gpu_windows.py."""
import struct

import numpy as np
import pytest

import orc
import py_oracle
from hbam import synth

CONTIG_LEN = [249250621, 243199373, 198022430, 191154276, 180915260, 171115067, 159138663, 146364022, 141213431,
              135534747, 135006516, 133851895, 115169878, 107349540, 102531392, 90354753, 81195210, 78077248,
              59128983, 63025520, 48129895, 51304566, 155270560, 59373566, 16571]


def test_test_bam_passes_strict(test_bam):
    s = orc.Stream(test_bam)
    rc, r = s.decode_all()
    assert rc == 0 and len(r["key"]) == 2277


def _records(**kw):
    d, _ = synth.make_bam(**kw)
    s = orc.Stream(d, stringency=orc.SILENT)
    rc, r = s.decode_all()
    assert rc == 0
    u = s.data
    out = []
    for i in range(len(r["key"])):
        p = int(r["offset"][i])
        bs = struct.unpack_from("<i", u, p)[0]
        out.append(bytearray(u[p:p + 4 + bs]))
    return out


def _mutate(rec, rng):
    r = bytearray(rec)
    lrn, ncig = r[12], struct.unpack_from("<H", r, 16)[0]
    k = rng.integers(0, 10)
    if k == 0:
        struct.pack_into("<H", r, 18, struct.unpack_from("<H", r, 18)[0] ^ (1 << int(rng.integers(0, 12))))
    elif k == 1:
        r[13] = int(rng.integers(0, 256))
    elif k == 2:
        struct.pack_into("<H", r, 14, int(rng.integers(0, 37450)))
    elif k == 3 and ncig:
        j = int(rng.integers(0, ncig))
        c = struct.unpack_from("<I", r, 36 + lrn + 4 * j)[0]
        c = (c & ~15) | int(rng.integers(0, 10)) if rng.random() < 0.7 else (int(rng.integers(0, 200)) << 4) | (c & 15)
        struct.pack_into("<I", r, 36 + lrn + 4 * j, c)
    elif k == 4:
        struct.pack_into("<i", r, 24, int(rng.choice([-1, 0, 3, 24])))
    elif k == 5:
        struct.pack_into("<i", r, 28, int(rng.choice([-1, 0, 5, 20000, 300000000])))
    elif k == 6:
        struct.pack_into("<i", r, 8, int(rng.choice([-1, 0, 16570, 16571, 20000])))
    elif k == 7:
        struct.pack_into("<i", r, 4, int(rng.choice([-1, 0, 24])))
    elif k == 8:
        struct.pack_into("<i", r, 20, int(rng.choice([0, 149, 151, 100000])))
    else:
        r[12] = int(rng.choice([0, 1, lrn + 3]))
    return bytes(r)


@pytest.mark.parametrize("kw", [dict(n_records=400), dict(n_records=12, mode="long"),
                                dict(n_records=200, all_unmapped=True)])
def test_two_restatements_agree_on_mutations(kw):
    recs = _records(**kw)
    rng = np.random.default_rng(11)
    seen = {True: 0, False: 0}
    for t in range(3000):
        rec = _mutate(recs[int(rng.integers(0, len(recs)))], rng)
        if rng.random() < 0.3:
            rec = _mutate(rec, rng)
        for strict in (True, False):
            for rl in (None, CONTIG_LEN):
                a = orc.record_invalid(rec, 25, rl, strict)
                b = py_oracle.record_invalid(rec, 25, rl, strict)
                assert a == b, (t, strict, rl is None, rec[:40].hex())
                seen[a] += 1
    assert seen[True] > 1000 and seen[False] > 1000


def test_valid_synthetic_records_pass():
    for kw in (dict(n_records=2000), dict(n_records=30, mode="long"), dict(n_records=40, mode="long", all_unmapped=True)):
        for rec in _records(**kw):
            assert not orc.record_invalid(bytes(rec), 25, CONTIG_LEN, True)
            assert not py_oracle.record_invalid(bytes(rec), 25, CONTIG_LEN, True)


def test_empty_read_needs_fz_or_cq_cs():
    rec = _records(n_records=60, all_unmapped=True)[0]
    lrn, ncig = rec[12], struct.unpack_from("<H", rec, 16)[0]
    lseq = struct.unpack_from("<i", rec, 20)[0]
    head = bytearray(rec[:36 + lrn + 4 * ncig])
    struct.pack_into("<i", head, 20, 0)  # l_seq 0: no seq / qual
    for aux, bad in ((b"", True), (b"FZB" + b"S" + struct.pack("<i", 0), False),
                     (b"CQZab\0CSZcd\0", False), (b"CQZ\0CSZcd\0", True), (b"RGZx\0", True)):
        r = bytearray(head + aux)
        struct.pack_into("<i", r, 0, len(r) - 4)
        assert orc.record_invalid(bytes(r), 25, None, True) == bad
        assert py_oracle.record_invalid(bytes(r), 25, None, True) == bad
    assert lseq > 0


def test_stringency_levels_in_oracle_decode():
    d, _ = synth.make_bam(3000)
    s = orc.Stream(d, stringency=orc.SILENT)
    rc, r = s.decode_all()
    u = bytearray(s.data)
    p = int(r["offset"][1700])
    struct.pack_into("<H", u, p + 14, 1)  # wrong bin: a STRICT-only error
    from test_gpu_windows import recompress
    bad = recompress(s, bytes(u))
    for st, want_rc, want_n in ((orc.STRICT, 1, 1700), (orc.LENIENT, 0, 3000), (orc.SILENT, 0, 3000)):
        rc, got = orc.Stream(bad, stringency=st).decode_all()
        assert rc == want_rc and len(got["key"]) == want_n
