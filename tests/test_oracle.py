"""CPU: the oracle (oracle/hbam_oracle.c) against the reference's own pins,
the committed golden vectors and the independent Python restatement."""
import hashlib
import os

import numpy as np
import pytest

import orc
import py_oracle
from conftest import GOLDEN, golden_path


def test_first_record_voff_pin(test_bam, golden):
    # TestBAMSplitGuesser.java:17-23: guessNextBAMRecordStart(0, ..) == first record voff
    s = orc.Stream(test_bam)
    assert s.first_record_voff == 0x196A == golden["first_record_voff"]
    assert s.guess_record_start(0, 3 * 0xFFFF + 0xFFFE) == 0x196A


def test_records_match_golden(test_bam):
    s = orc.Stream(test_bam)
    rc, r = s.decode_all()
    assert rc == 0
    g = np.load(golden_path("test.bam.records.npz"))
    for k in g.files:
        np.testing.assert_array_equal(r[k], g[k], err_msg=k)
    assert hashlib.sha256(r["key"].tobytes()).hexdigest().startswith("9cec72cb")


@pytest.mark.parametrize("g", [1, 2, 10, 4096])
def test_splitting_index_golden(test_bam, g):
    s = orc.Stream(test_bam)
    want = open(golden_path(f"test.bam.g{g}.splitting-bai"), "rb").read()
    got = s.splitting_index(g)
    assert got == want
    # TestSplittingBAMIndexer.java:31-32: bamSize() == file length
    assert int.from_bytes(got[-8:], "big") >> 16 == len(test_bam)
    n = {1: 2279, 2: 1140, 10: 229, 4096: 2}[g]
    assert len(got) // 8 == n


def test_index_matches_processAlignment_semantics(test_bam):
    # TestSplittingBAMIndexer: index() and processAlignment() give equal SplittingBAMIndex sets
    s = orc.Stream(test_bam)
    rc, r = s.decode_all()
    for g in (2, 10, 4096):
        ent = []
        for c, v in enumerate(r["voff"]):
            if c == 0 or (c + 1) % g == 0:
                ent.append(int(v))
        ent.append(len(test_bam) << 16)
        idx = s.splitting_index(g)
        got = {int.from_bytes(idx[i:i + 8], "big") for i in range(0, len(idx), 8)}
        assert got == set(ent)


def test_bgzf_text_fixtures(golden):
    for f, t in golden["bgzf_text"].items():
        data = open(golden_path(f), "rb").read()
        x = orc.Stream(data, check_crc=True, parse_header=False)
        assert hashlib.sha256(x.data).hexdigest() == t["sha256"] and len(x.data) == t["len"]
        assert [int(b["coff"]) for b in x.blocks] == t["coffs"]


@pytest.mark.parametrize("f,first,last", [("test.vcf.bgzf.gz", 821, 821), ("HiSeq.10000.vcf.bgzf.gz", 16688, 509222)])
def test_bgzf_split_guesser_pins(f, first, last):
    # TestBGZFSplitGuesser.java:32-63
    data = open(golden_path(f), "rb").read()
    bnd, start = [], 1
    while True:
        ns = orc.guess_next_bgzf_block_start(data, start, len(data))
        if ns == len(data):
            break
        bnd.append(ns)
        start = ns + 1
    assert bnd[0] == first and bnd[-1] == last and bnd[-1] == len(data) - 28


def test_guesser_golden(test_bam, golden):
    s = orc.Stream(test_bam)
    for beg, end, want in golden["guesses"]:
        assert s.guess_record_start(beg, end) == want, (beg, end)


def test_split_planning_golden(test_bam, golden):
    s = orc.Stream(test_bam)
    sbi = s.splitting_index(4096)
    for p in golden["plans"]:
        assert [list(x) for x in s.get_splits(p["starts"], p["lengths"], sbi)] == p["indexed"]
        assert [list(x) for x in s.get_splits(p["starts"], p["lengths"], None)] == p["probabilistic"]


def test_murmur_c_vs_python():
    rng = np.random.default_rng(7)
    for n in list(range(0, 40)) + [300, 331, 1000]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 1, -5):
            assert orc.murmurhash3(b, seed) == py_oracle.murmurhash3(b, seed)


def test_key_edge_cases():
    # BAMRecordReader.java:81-121 worked examples
    assert orc.get_key(1, 99, 0, b"") == 0x0000000100000063
    assert orc.get_key(3, -1, 0, b"") == -1          # pos -1 mapped: sign-extended
    k = orc.get_key(0, 5, 4, b"abc")                  # unmapped -> murmur branch
    h = py_oracle.murmurhash3(b"abc") & 0xFFFFFFFF
    h = h - (1 << 32) if h >> 31 else h
    assert k == ((0x7FFFFFFF << 32) | (h & 0xFFFFFFFFFFFFFFFF)) - (1 << 64) * (h < 0)
    assert orc.get_key(-1, -1, 0, b"xyz") == py_oracle.get_key(-1, -1, 0, b"xyz")
    assert orc.get_key(2, -2, 0, b"q") == py_oracle.get_key(2, -2, 0, b"q")  # start < 0 -> hash


@pytest.mark.parametrize("kw", [dict(n_records=1500), dict(n_records=60, mode="long"), dict(n_records=800, level=0),
                                dict(n_records=800, strategy="fixed"), dict(n_records=400, all_unmapped=True),
                                dict(n_records=1500, mode="wgs")])
def test_oracle_vs_python_synthetic(kw):
    from hbam import synth
    d, _ = synth.make_bam(**kw)
    s = orc.Stream(d, check_crc=True)
    rc, r = s.decode_all()
    assert rc == 0
    pr = py_oracle.records(d)
    assert [k for _, k in pr] == [int(x) for x in r["key"]]
    assert [v for v, _ in pr] == [int(x) for x in r["voff"]]
    for g in (1, 7, 4096):
        assert s.splitting_index(g) == py_oracle.splitting_index(d, g)


def test_scan_digests_are_order_sensitive_and_compose():
    """orc_scan's key / voff digests (the 60 GB bench parity): equal to the
    Horner digest of the single-threaded oracle's columns at any thread count,
    composable over consecutive runs, and changed by swapping two records --
    which the xor / sum digests cannot see."""
    from hbam import synth
    data, _ = synth.make_bam(6000, as_numpy=True, block_payload=8192)
    rc, want = orc.Stream(data.tobytes()).decode_all()
    assert rc == 0
    keys = want["key"].astype(np.uint64)
    kd, vd = orc.digest(keys), orc.digest(want["voff"])
    for threads in (1, 3, 8):
        r, _ = orc.scan(data, threads=threads)
        assert (r["records"], r["key_digest"], r["voff_digest"]) == (len(keys), kd, vd)
    ri, _ = orc.scan(data, threads=4, mode="index")
    assert ri["voff_digest"] == vd
    a = len(keys) // 3
    assert orc.digest_concat([(a, orc.digest(keys[:a])), (len(keys) - a, orc.digest(keys[a:]))]) == (len(keys), kd)
    sw = keys.copy()
    i = int(np.nonzero(sw[:-1] != sw[1:])[0][0])
    sw[[i, i + 1]] = sw[[i + 1, i]]
    assert orc.digest(sw) != kd
    d, k, v = orc.scan_records(data, len(keys), threads=5)
    assert d["rc"] == 0
    np.testing.assert_array_equal(k, want["key"])
    np.testing.assert_array_equal(v, want["voff"])


def test_scan_field_and_rest_digests():
    """orc_scan's per-field digests and rest crc32 (the at-scale parity of
    tests/test_gpu_large.py): equal, at any thread count, to the digests of
    the single-threaded oracle's columns and to the crc32 of its rests in
    record order; the vectorized digest equals the scalar one."""
    import zlib
    from hbam import synth
    data, _ = synth.make_bam(5000, as_numpy=True, block_payload=8192)
    s = orc.Stream(data.tobytes())
    rc, want = s.decode_all()
    assert rc == 0
    u = s.data
    rests = b"".join(u[o + 36:o + 36 + n] for o, n in zip(want["offset"].tolist(), want["rest_len"].tolist()))
    for threads in (1, 4):
        r, _ = orc.scan(data, threads=threads)
        assert r["rc"] == 0
        for f in orc._ScanResult.FIELDS:
            assert r["field_digest"][f] == orc.digest_np(want[f])[1], f
        assert r["rest_bytes"] == len(rests) and r["rest_crc"] == zlib.crc32(rests)
    v = want["tlen"]
    assert orc.digest_np(v)[1] == orc.digest([int(x) & ((1 << 64) - 1) for x in v.astype(np.int64)])


def test_synthetic_reads_at_a_contig_end_are_valid():
    """The generator's model at 80 M records (bench.py's weak N x C2 leg at
    N = 8) walks past chr1's end: the reads placed there, and their mates'
    starts, stay inside the contig (STRICT: a mate start past the reference
    length is a SAMFormatException)."""
    from hbam import synth
    n, end = 80_000_000, 249_250_621 // 5  # model span: 5 bp per mapped read
    h, _ = synth.make_bam_segment(n, 0, 0, with_header=True, eof_block=False)
    seg, _ = synth.make_bam_segment(n, end - 1000, end + 1000, with_header=False, eof_block=True)
    s = orc.Stream(np.concatenate([h, seg]).tobytes())
    rc, got = s.decode_span(h.nbytes << 16, (1 << 64) - 1)
    assert rc == 0 and len(got["key"]) == 2000
    assert (got["ref_id"] == 0).any() and (got["ref_id"] == 1).any()  # the walk crosses chr1's end
