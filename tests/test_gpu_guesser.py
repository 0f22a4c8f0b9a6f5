"""The BAMSplitGuesser drop-in (hbam.BAMSplitGuesser, the Python mirror of
java/.../GpuBAMSplitGuesser.java) reading through a positioned-read callback
over a seekable stream -- no mapping of the file, only the bytes each guess
needs -- against TestBAMSplitGuesser.java:17-23 (the first record of test.bam
at 0x196a), the golden per-block guesses, and the oracle's guesser with the
three-argument constructor's separate header stream (BAMSplitGuesser.java:
93-103: the header's dictionary bounds the refIDs a guessed record holds)."""
import io
import struct
import zlib

import pytest

import hbam
import orc
from conftest import golden_path

pytestmark = pytest.mark.gpu
MAX_BYTES_READ = 3 * 0xffff + 0xfffe


class CountingFile(io.FileIO):
    """A file read only through seek + read, with the bytes read counted."""

    def __init__(self, path):
        super().__init__(path, "r")
        self.nread = 0

    def read(self, n=-1):
        b = super().read(n)
        self.nread += len(b)
        return b


def test_reference_case_first_record():
    # TestBAMSplitGuesser.java:17-23: new BAMSplitGuesser(ss, conf)
    #   .guessNextBAMRecordStart(0, 3 * 0xffff + 0xfffe) == the first record
    with CountingFile(golden_path("test.bam")) as ss, hbam.BAMSplitGuesser(ss) as g:
        assert g.guessNextBAMRecordStart(0, MAX_BYTES_READ) == 0x196A


def test_golden_guesses_one_call_each(golden):
    size = len(open(golden_path("test.bam"), "rb").read())
    with CountingFile(golden_path("test.bam")) as ss, hbam.BAMSplitGuesser(ss) as g:
        n0 = ss.nread
        for beg, end, want in golden["guesses"]:
            assert g.guessNextBAMRecordStart(beg, end) == want, (beg, end)
        # each guess reads about its MAX_BYTES_READ window, never the file
        # over and over (the windows of nearby points overlap)
        assert ss.nread - n0 <= len(golden["guesses"]) * (MAX_BYTES_READ + (1 << 17)) + size


def _bam_with_refs(test_bam: bytes, k: int) -> bytes:
    """test.bam's header with only its first k references (binary list and
    @SQ lines, which htsjdk requires to agree), as a header-only BAM (what
    SAMHeaderReader reads from the header stream)."""
    s = orc.Stream(test_bam)
    u = bytes(s.data)
    l_text = struct.unpack_from("<i", u, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", u, p)[0]
    assert 0 <= k <= n_ref
    q = p + 4
    for _ in range(k):
        ln = struct.unpack_from("<i", u, q)[0]
        q += 4 + ln + 4
    lines, sq = [], 0
    for ln in u[8:p].rstrip(b"\0").split(b"\n"):
        if ln.startswith(b"@SQ"):
            sq += 1
            if sq > k:
                continue
        lines.append(ln)
    text = b"\n".join(lines)
    hdr = u[:4] + struct.pack("<i", len(text)) + text + struct.pack("<i", k) + u[p + 4:q]
    return orc.bgzf_compress(hdr, [len(hdr)], level=5, eof=True)


@pytest.mark.parametrize("k", [0, 1, None])
def test_header_stream_bounds_the_refids(test_bam, golden, tmp_path, k):
    n_ref = golden["n_ref"]
    k = n_ref if k is None else min(k, n_ref)
    hp = tmp_path / f"header_{k}.bam"
    hp.write_bytes(_bam_with_refs(test_bam, k))
    s = orc.Stream(test_bam)
    with CountingFile(golden_path("test.bam")) as ss, open(hp, "rb") as hs, hbam.BAMSplitGuesser(ss, hs) as g:
        for beg, end, _ in golden["guesses"][:24]:
            assert g.guessNextBAMRecordStart(beg, end) == s.guess_record_start(beg, end, header_n_ref=k), (beg, k)


def test_not_a_bam_stream_is_rejected(tmp_path):
    p = tmp_path / "plain.gz"
    p.write_bytes(zlib.compress(b"not a BAM file" * 1000))
    with open(p, "rb") as ss, pytest.raises(hbam.HbamError):
        hbam.BAMSplitGuesser(ss)
