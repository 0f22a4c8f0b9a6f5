"""The record pass's edge paths (Pipeline::decode_span_pos):
  (a) an early stop that is not an error, with records listed after it:
      [htsjdk] an empty BGZF block right after an exhausted one reads as EOF,
      so the reader stops mid-file, and when the blocks after it start at a
      record (a chain the walks follow) the fused check + output launch
      (k_rec_check_out) lists records there too.  The span ends at the first
      stop: those records are dropped (before round 5 a fallback rescanned
      the counts and kept them: 5,808 records where the reference reads
      3,000);
  (b) a list overflow: SplittingBAMIndexer.index (SplittingBAMIndexer.java:
      262-287) skips block_size bytes whatever they are, so block_size-0
      records are 4 bytes long and a 64 KiB block holds more of them than a
      list has room for (kListCap, sized for >= 36-byte reader records): the
      per-block walks count and emit the records instead (k_rec_count,
      k_rec_emit), and stop at EOF the same way.
Each case is checked against the oracle, and hbam_pipeline_counters shows
the path that ran."""
import struct

import numpy as np
import pytest

import hbam
import orc
from hbam import synth
from test_gpu_parity import assert_same_records

pytestmark = pytest.mark.gpu
ALL = (1 << 64) - 1


def test_records_after_an_eof_block_take_the_separate_launches():
    d1, _ = synth.make_bam(3000, eof_block=True)
    d2, _ = synth.make_bam(3000, seed=99, eof_block=False)
    s2 = orc.Stream(d2)
    # file 2's records re-cut into blocks that start at its first record, so
    # that the chain goes on through them past file 1's EOF block: the reader
    # stops at the empty block (no error), and the walks list records after it
    recs = bytes(s2.data)[s2.header_end:]
    lens = [min(65280, len(recs) - a) for a in range(0, len(recs), 65280)]
    data = d1 + orc.bgzf_compress(recs, lens, level=5, eof=True)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0 and len(want["key"]) == 3000
    with hbam.BamFile(data, window_bytes=1 << 30) as f:
        c0 = f.pipeline_counters()
        got = f.decode_all()
        assert_same_records(got, want)
        c1 = f.pipeline_counters()
        assert c1["records_after_stop"] > c0["records_after_stop"]
        st = f.decode_span_device(f.header()["first_record_voff"], ALL)
        assert st["records"] == 3000 and st["status"] == 0
        assert f.splitting_index(5) == s.splitting_index(5)


@pytest.mark.parametrize("eof_mid", [False, True])
@pytest.mark.parametrize("g", [1, 7, 4096])
def test_indexer_list_overflow_takes_the_separate_launches(g, eof_mid):
    d, _ = synth.make_bam(4000, seed=5)
    s0 = orc.Stream(d)
    u = bytes(s0.data)
    h = s0.header_end
    # the first 1500 records, 40,000 block_size-0 records (160 KB: more than
    # kListCap per 64 KiB block), then the rest
    q, n = h, 0
    while n < 1500:
        q += 4 + struct.unpack_from("<i", u, q)[0]
        n += 1
    payload = u[:q] + b"\0" * (4 * 40000) + u[q:]
    lens = [min(65280, len(payload) - a) for a in range(0, len(payload), 65280)]
    data = orc.bgzf_compress(payload, lens, level=5, eof=True)
    if eof_mid:  # an EOF block mid-file, then records from a block start: the index ends at it
        d2, _ = synth.make_bam(2000, seed=8, eof_block=False)
        s2 = orc.Stream(d2)
        recs = bytes(s2.data)[s2.header_end:]
        data += orc.bgzf_compress(recs, [min(65280, len(recs) - a) for a in range(0, len(recs), 65280)], level=5)
    s = orc.Stream(data)
    want = s.splitting_index(g)
    with hbam.BamFile(data) as f:
        c0 = f.pipeline_counters()
        assert f.splitting_index(g) == want
        assert f.pipeline_counters()["record_fallbacks"] > c0["record_fallbacks"]


def _with_false_start(n=3000, at=(1000,), seed=3):
    """A C2-like BAM whose records `at` each carry, as their last tag (B:c),
    the bytes of another whole record, and a BGZF block that starts exactly
    there: the block's first plausible record start is that embedded copy,
    whose chain runs on into the true next record."""
    d, _ = synth.make_bam(n, seed=seed)
    s0 = orc.Stream(d)
    u = bytes(s0.data)
    h = s0.header_end
    starts, q = [], h
    while q < len(u):
        starts.append(q)
        q += 4 + struct.unpack_from("<i", u, q)[0]
    out, cuts, prev = bytearray(u[:h]), [], h
    for r in sorted(at):
        a, b = starts[r], starts[r + 1]
        donor = u[starts[n - 1 - r]:starts[n - r]] if n - r < len(starts) else u[starts[n - 1 - r]:]
        out += u[prev:a]
        body = bytearray(u[a + 4:b]) + b"XXBc" + struct.pack("<i", len(donor))
        cuts.append(len(out) + 4 + len(body))  # the embedded copy's first byte
        body += donor
        out += struct.pack("<i", len(body)) + body
        prev = b
    out += u[prev:]
    lens, p = [], 0
    for c in cuts + [len(out)]:
        while c - p > 65280:
            lens.append(65280)
            p += 65280
        if c > p:
            lens.append(c - p)
            p = c
    return orc.bgzf_compress(bytes(out), lens, level=5, eof=True)


@pytest.mark.parametrize("at", [(1000,), (700, 1400, 2100)])
def test_false_start_at_a_block_start_is_rewalked(at):
    """(c) the link check's re-walk round: the speculative list bound queued
    with the first link check is discarded and recomputed after it."""
    data = _with_false_start(at=at)
    s = orc.Stream(data)
    rc, want = s.decode_all()
    assert rc == 0 and len(want["key"]) == 3000
    with hbam.BamFile(data, window_bytes=1 << 30) as f:
        c0 = f.pipeline_counters()
        got = f.decode_all()
        assert_same_records(got, want)
        c1 = f.pipeline_counters()
        assert c1["link_rewalks"] + c1["link_fallbacks"] > c0["link_rewalks"] + c0["link_fallbacks"]
        st = f.decode_span_device(f.header()["first_record_voff"], ALL)
        assert st["records"] == 3000 and st["status"] == 0
        assert st["first_voff"] == want["voff"][0] and st["last_voff"] == want["voff"][-1]
        assert f.splitting_index(5) == s.splitting_index(5)
