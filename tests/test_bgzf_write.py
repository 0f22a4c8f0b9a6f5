"""BGZF write path: [htsjdk] BlockCompressedOutputStream
(deflateBlock + writeGzipBlock; the compressor BAMRecordWriter.java:131-149
writes through) on the GPU, byte-identical to zlib 1.2.11.

Pins: the reference's own fixtures are recompressed byte for byte from their
inflated payloads -- test.bam (htsjdk-written, 65498-byte blocks) at level 5,
HiSeq.10000.vcf.bgzf.gz (bgzip, 65280-byte blocks) at level 6 -- first by the
oracle (system zlib, the library java.util.zip.Deflater wraps), then by the
GPU.  The host-compiled restatement (hbam_deflate.h) is compared with zlib by
lib/deflate_check in both Deflater lifecycles (reset per block / fresh per
block).  At full size: recompressing a synthetic C2-like BAM (zlib level 5,
fresh stream per block) reproduces the file."""
import os
import subprocess
import zlib

import numpy as np
import pytest

import orc
from conftest import ROOT, golden_path

CHECK = os.path.join(ROOT, "hadoop-bam_amd", "lib", "deflate_check")


def split_bgzf(data):
    """(payload bytes, ISIZE list, has EOF terminator) of a BGZF file."""
    p, lens, pay = 0, [], []
    while p < len(data):
        bs = int.from_bytes(data[p + 16:p + 18], "little") + 1
        u = zlib.decompressobj(-15).decompress(data[p + 18:p + bs - 8])
        lens.append(len(u))
        pay.append(u)
        p += bs
    eof = bool(lens) and lens[-1] == 0 and data.endswith(bytes.fromhex("1b0003000000000000000000"))
    if eof:
        lens = lens[:-1]
    return b"".join(pay), lens, eof


FIXTURES = [("test.bam", 5), ("HiSeq.10000.vcf.bgzf.gz", 6), ("test.vcf.bgzf.gz", 5), ("test.bgzf.bcf", 5)]


@pytest.mark.parametrize("name,level", FIXTURES)
def test_oracle_recompresses_reference_fixtures(name, level):
    data = open(golden_path(name), "rb").read()
    u, lens, eof = split_bgzf(data)
    assert orc.bgzf_compress(u, lens, level=level, eof=eof) == data


def test_oracle_htsjdk_fallback_and_edges():
    rng = np.random.default_rng(7)
    noise = rng.integers(0, 256, 65498, dtype=np.uint8).tobytes()
    out = orc.bgzf_compress(noise, [65498], level=5, eof=False)
    # incompressible: level-5 output would exceed the 65518-byte buffer -> one stored block
    assert out[18] == 1 and int.from_bytes(out[19:21], "little") == 65498 and out[23:23 + 65498] == noise
    assert zlib.decompressobj(-15).decompress(out[18:-8]) == noise
    empty = orc.bgzf_compress(b"", [], level=5, eof=True)
    assert len(empty) == 28


def test_host_restatement_matches_zlib(tmp_path):
    assert os.path.exists(CHECK), "build() makes hadoop-bam_amd/lib/deflate_check"
    r = subprocess.run([CHECK], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-2000:]
    u, _, _ = split_bgzf(open(golden_path("test.bam"), "rb").read())
    f = tmp_path / "test.bam.u"
    f.write_bytes(u)
    r = subprocess.run([CHECK, str(f)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-2000:]


# ---------------------------------------------------------------- GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("name,level", FIXTURES)
def test_gpu_recompresses_reference_fixtures(name, level):
    import hbam
    data = open(golden_path(name), "rb").read()
    u, lens, eof = split_bgzf(data)
    assert hbam.bgzf_compress(u, block_lens=lens, level=level, eof=eof) == data


def _cases():
    rng = np.random.default_rng(0x5A)
    acgt = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 600000)].tobytes()
    runs = bytes((i // 3000) & 0xFF for i in range(400000))
    noise = rng.integers(0, 256, 300000, dtype=np.uint8).tobytes()
    u, _, _ = split_bgzf(open(golden_path("test.bam"), "rb").read())
    return {"acgt": acgt, "runs": runs, "noise": noise, "bam": u}


@pytest.mark.gpu
@pytest.mark.parametrize("level", [0, 1, 2, 3, 4, 5, 6, 9])
def test_gpu_vs_oracle_levels(level):
    import hbam
    for name, d in _cases().items():
        for bs in (65498, 65280, 65536, 4097):
            if (name == "noise" or level == 0) and bs == 65536:
                continue  # no stored fallback fits (test_gpu_ragged_blocks_and_empty)
            n = len(d)
            lens = [min(bs, n - p) for p in range(0, n, bs)]
            got = hbam.bgzf_compress(d, block_size=bs, level=level, eof=True)
            assert got == orc.bgzf_compress(d, lens, level=level, eof=True), (name, bs, level)


@pytest.mark.gpu
def test_gpu_ragged_blocks_and_empty():
    import hbam
    d = _cases()["bam"]
    lens = [0, 1, 2, 3, 258, 65273, 65274, 65275, 65536, 1000, 0, 65498]
    payload = (d * 2)[:sum(lens)]
    assert hbam.bgzf_compress(payload, block_lens=lens, level=5) == orc.bgzf_compress(payload, lens, level=5)
    assert hbam.bgzf_compress(b"", level=5, eof=True) == orc.bgzf_compress(b"", [], level=5, eof=True)
    noise = np.random.default_rng(3).integers(0, 256, 65536, dtype=np.uint8).tobytes()
    with pytest.raises(hbam.HbamError):  # stored fallback cannot fit 65536 + 5 bytes
        hbam.bgzf_compress(noise, block_size=65536, level=5)
    for bs in (65498, 65513):  # the NO_COMPRESSION fallback (and its last size that fits)
        assert hbam.bgzf_compress(noise[:bs], block_size=bs, level=5) == orc.bgzf_compress(noise[:bs], [bs], level=5)


@pytest.mark.gpu
def test_gpu_recompress_synthetic_bam_full_roundtrip():
    """C2-shaped file (200k records, zlib level 5, fresh stream per block):
    inflate on the GPU, then recompress the resident stream with the same
    block boundaries -> the original bytes."""
    import hbam
    from hbam import synth
    data, info = synth.make_bam(200000, seed=0x42475A57, as_numpy=True)
    g = hbam.Gpu(0)
    try:
        g.load(data)
        g.run()
        ms, n = g.bgzf_compress(level=5, eof=False)
        got = g.fetch_compressed(0, n)
        assert n == data.nbytes and np.array_equal(got, data)
    finally:
        g.close()


@pytest.mark.gpu
def test_gpu_multi_batch_framing(monkeypatch):
    """More blocks than one batch of arenas: offsets continue across batches."""
    import hbam
    d = _cases()["acgt"] + _cases()["bam"]
    lens = [min(4097, len(d) - p) for p in range(0, len(d), 4097)]
    want = orc.bgzf_compress(d, lens, level=5, eof=True)
    monkeypatch.setenv("HBAM_DFL_MAX_LANES", "37")
    assert hbam.bgzf_compress(d, block_lens=lens, level=5, eof=True) == want
