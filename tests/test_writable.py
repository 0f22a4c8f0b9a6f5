"""SAMRecordWritable codec (SAMRecordWritable.java:55-68).

write()      = [htsjdk] BAMRecordCodec.encode of the BAMRecord BAMRecordReader
               hands out: the record re-serialized from its fields (indexBin 0
               when refID < 0, rest verbatim).
readFields() = [htsjdk] BAMRecordCodec.decode (LazyBAMRecordFactory, no header)
               per framed value.

CPU tests pin the C oracle against the independent Python restatement and the
reference's own fixture (test.bam); GPU tests compare libhbam (through the C
ABI) with the oracle, bit-exact.
"""
import struct

import numpy as np
import pytest

import hbam
import orc
import py_oracle
from hbam import synth

FIELDS = ["ref_id", "pos", "l_seq", "next_ref_id", "next_pos", "tlen", "l_read_name", "mapq", "bin",
          "n_cigar", "flag", "key", "rest_len"]


def _oracle_encode(data):
    s = orc.Stream(data)
    rc, enc, offs = s.writable_encode_span(s.first_record_voff, (1 << 64) - 1)
    assert rc == 0
    return s, enc, offs


def _record(ref=-1, pos=-1, bin_=4680, flag=4, name=b"r1", seq_len=3, aux=b"", bs_delta=0):
    rest = name + b"\0" + bytes((seq_len + 1) // 2) + bytes([30] * seq_len) + aux
    bs = 32 + len(rest) + bs_delta
    return struct.pack("<iiiBBHHHiiii", bs, ref, pos, len(name) + 1, 0, bin_, 0, flag, seq_len, -1, -1, 0) + rest


# ---------------------------------------------------------------- CPU (oracle)

def test_oracle_encode_test_bam_matches_python_and_raw(test_bam):
    s, enc, offs = _oracle_encode(test_bam)
    assert enc == py_oracle.writable_encode(test_bam)
    # test.bam: every record refID 0, so write() reproduces the record bytes
    assert enc == s.data[s.header_end:s.header_end + len(enc)]
    assert len(offs) == 2277 + 1 and offs[-1] == len(enc)


def test_oracle_encode_unplaced_bin_zeroed():
    data, _ = synth.make_bam(3000, seed=0x57524954)
    s, enc, offs = _oracle_encode(data)
    assert enc == py_oracle.writable_encode(data)
    rc, cols = s.decode_all()
    unplaced = np.nonzero(cols["ref_id"] < 0)[0]
    assert len(unplaced) > 0 and np.all(cols["bin"][unplaced] == 4680)
    for i in unplaced[:20]:
        assert enc[int(offs[i]) + 14:int(offs[i]) + 16] == b"\0\0"
    placed = np.nonzero(cols["ref_id"] >= 0)[0][:20]
    for i in placed:
        assert struct.unpack_from("<H", enc, int(offs[i]) + 14)[0] == cols["bin"][i]


def test_oracle_readfields_roundtrip_and_errors(test_bam):
    s, enc, offs = _oracle_encode(test_bam)
    rc, want = s.decode_all()
    rc2, got = orc.writable_decode(enc, offs[:-1])
    assert rc2 == 0
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)
    assert np.all(got["voff"] == np.uint64(2**64 - 1))
    # value 1 cut short / block_size < 32 / fewer than 4 bytes
    cut = enc[:int(offs[2]) - 5]
    rc, got = orc.writable_decode(cut, offs[:2])
    assert rc == orc_status("TRUNC") and len(got["key"]) == 1
    bad = bytearray(enc[:int(offs[2])])
    struct.pack_into("<i", bad, int(offs[1]), 31)
    rc, got = orc.writable_decode(bytes(bad), offs[:2])
    assert rc == orc_status("FORMAT") and len(got["key"]) == 1
    rc, got = orc.writable_decode(b"\1\0\0", [0])
    assert rc == orc_status("TRUNC") and len(got["key"]) == 0


def orc_status(name):
    return {"FORMAT": 1, "TRUNC": 2, "ARG": 3}[name]


def test_codec_fails_loudly_without_gpu():
    if hbam.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(hbam.HbamError) as e:
        hbam.Codec(0)
    assert e.value.code == hbam.E_DEVICE


# ---------------------------------------------------------------- GPU (parity)

@pytest.mark.gpu
@pytest.mark.parametrize("case", ["test.bam", "short", "long"])
def test_gpu_encode_matches_oracle(test_bam, case):
    if case == "test.bam":
        data = test_bam
    else:
        data, _ = synth.make_bam(4000 if case == "short" else 60, mode=case, seed=0x57524955)
    _, want, want_offs = _oracle_encode(data)
    with hbam.BamFile(data) as f:
        f.decode_all()
        got, offs = f.encode_writables()
    assert got == want
    np.testing.assert_array_equal(offs, want_offs)


@pytest.mark.gpu
def test_gpu_encode_split_spans_concatenate(test_bam):
    """Encodings of consecutive splits concatenate to the whole file's."""
    _, want, _ = _oracle_encode(test_bam)
    with hbam.BamFile(test_bam) as f:
        splits = f.get_splits([0, 100000, 200000], [100000, 100000, len(test_bam) - 200000])
        parts = []
        for vs, ve in splits:
            f.decode_span(vs, ve)
            parts.append(f.encode_writables()[0])
    assert b"".join(parts) == want


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["short", "long"])
def test_gpu_readfields_matches_oracle(mode):
    # long: ONT-like unmapped records take the deferred k_long_hash key path
    data, _ = synth.make_bam(5000 if mode == "short" else 80, mode=mode, all_unmapped=mode == "long",
                             seed=0x57524956)
    _, enc, offs = _oracle_encode(data)
    # frame with gaps, as a shuffle stream would (a vint length before each value)
    gap = 3
    buf = bytearray()
    framed = []
    for i in range(len(offs) - 1):
        buf += b"\x7f" * gap
        framed.append(len(buf))
        buf += enc[int(offs[i]):int(offs[i + 1])]
    rc, want = orc.writable_decode(bytes(buf), framed)
    assert rc == 0
    with hbam.Codec(0) as c:
        got = c.decode_writables(bytes(buf), framed)
    assert got["status"] == 0
    for f in FIELDS + ["voff"]:
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)
    for i in range(0, len(framed), 97):
        a = got["data"][int(got["rest_off"][i]):int(got["rest_off"][i]) + int(got["rest_len"][i])]
        assert a == enc[int(offs[i]) + 36:int(offs[i + 1])]


@pytest.mark.gpu
def test_gpu_readfields_errors_match_oracle():
    recs = [_record(ref=0, pos=10, bin_=4681, flag=0), _record(), _record(aux=b"XYZ")]
    enc = b"".join(recs)
    offs = np.cumsum([0] + [len(r) for r in recs[:-1]]).astype(np.uint64)
    cases = [
        (enc, offs),                                    # clean
        (enc[:-2], offs),                               # last value short -> TRUNC
        (enc[:int(offs[1]) + 2] , offs[:2]),            # value 1 has no block_size -> TRUNC
        (enc[:int(offs[1])] + _record(bs_delta=-40), offs[:2]),  # block_size < 32 -> FORMAT
        (enc, np.array([0, len(enc) + 5], np.uint64)),  # framing outside buf -> ARG
    ]
    with hbam.Codec(0) as c:
        for buf, o in cases:
            rc, want = orc.writable_decode(buf, o)
            got = c.decode_writables(buf, o, raise_on_error=False)
            assert got["status"] == rc
            for f in FIELDS:
                np.testing.assert_array_equal(got[f], want[f], err_msg=f)


@pytest.mark.gpu
def test_gpu_device_encode_full_pipeline():
    """hbam_gpu_encode_writables (the bench entry) on a whole-file run."""
    data, info = synth.make_bam(20000, seed=0x57524957)
    _, want, _ = _oracle_encode(data)
    g = hbam.Gpu(0)
    try:
        g.load(data)
        g.run()
        ms, nb = g.encode_writables(iters=2)
        assert nb == len(want)
        assert g.fetch_encoded(0, nb) == want
    finally:
        g.close()
