"""Test infrastructure: the BAM index (.bai) side of split planning.

Only tests/ import this (never the product).  Two parts:

* `write_bai(data)` builds a .bai for a coordinate-sorted BAM, as htsjdk's
  BAMIndexer does for the linear index (16 kbp windows: each window's entry is
  the virtual offset of the first record overlapping it; windows no record
  overlaps take the last non-empty entry before them) plus per-bin chunk
  lists.  It makes the .bai fixtures the BAI split calculator reads; the
  reference writes its own with htsjdk (BAMTestUtil.writeBamFile), which
  cannot run here, so the fixtures' exact bytes are parity-unpinned -- the
  planner reads only the linear index, whose rule is the SAM spec's.

* `add_bai_splits(...)` restates BAMInputFormat.addBAISplits
  (src/main/java/org/seqdoop/hadoop_bam/BAMInputFormat.java:322-465) line by
  line, quirks included: a contig's last linear entry is never visited
  (`bin + 1 >= ctgBins` moves on first, :396-405), the last FileSplit is
  handled after the loop (:375-378, :447-459), a split with no linear entry
  inside it gets a guessed start and the previous split is cut there
  (:430-444).  Linear entries come from htsjdk's LinearIndex
  (getQueryResults(ctg).getLinearIndex(): size() = entries, get(i) =
  entry i; LinearBAMIndex.java:30-38); a contig with no bins has none.
"""
import struct

import numpy as np

import orc

LIDX_SHIFT = 14  # BAM_LIDX_SHIFT: 16 kbp linear windows


def _reg2bin(beg, end):
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def _ref_span(u, p):
    """(refID, pos, alignment end exclusive, flag) of the record at u[p]."""
    ref, pos = struct.unpack_from("<ii", u, p + 4)
    lrn = u[p + 12]
    ncig, flag = struct.unpack_from("<HH", u, p + 16)
    span = 0
    for k in range(ncig):
        c = struct.unpack_from("<I", u, p + 36 + lrn + 4 * k)[0]
        if (c & 15) in (0, 2, 3, 7, 8):  # M D N = X consume the reference
            span += c >> 4
    return ref, pos, pos + max(span, 1), flag


def write_bai(data: bytes) -> bytes:
    s = orc.Stream(data, stringency=orc.SILENT)
    rc, r = s.decode_all()
    if rc != 0:
        raise ValueError("BAM does not decode")
    u = s.data
    n_ref = s.n_ref
    lin = [dict() for _ in range(n_ref)]
    bins = [dict() for _ in range(n_ref)]
    voffs = [int(v) for v in r["voff"]]
    ends = voffs[1:] + [(len(data) << 16)]
    for i, p in enumerate(r["offset"]):
        ref, pos, end, flag = _ref_span(u, int(p))
        if ref < 0 or pos < 0:
            continue
        v = voffs[i]
        if flag & 4:  # placed unmapped: one position, samtools' window rule (BAMIndexer)
            w0 = max(pos - 1, 0) >> LIDX_SHIFT
            w1, end = w0, pos + 1
        else:
            w0, w1 = pos >> LIDX_SHIFT, (end - 1) >> LIDX_SHIFT
        for w in range(w0, w1 + 1):
            if w not in lin[ref]:
                lin[ref][w] = v
        b = _reg2bin(pos, end)
        ch = bins[ref].setdefault(b, [])
        if ch and ch[-1][1] == v:
            ch[-1][1] = ends[i]
        else:
            ch.append([v, ends[i]])
    out = bytearray(b"BAI\1")
    out += struct.pack("<i", n_ref)
    for ref in range(n_ref):
        out += struct.pack("<i", len(bins[ref]))
        for b in sorted(bins[ref]):
            out += struct.pack("<Ii", b, len(bins[ref][b]))
            for a, e in bins[ref][b]:
                out += struct.pack("<QQ", a, e)
        if lin[ref]:
            top = max(lin[ref])
            entries, last = [], 0
            for w in range(top + 1):
                last = lin[ref].get(w, last)
                entries.append(last)
        else:
            entries = []
        out += struct.pack("<i", len(entries))
        out += b"".join(struct.pack("<Q", e) for e in entries)
    return bytes(out)


def linear_index(bai: bytes):
    """Per reference, its linear index entries (empty for a reference with
    no bins) -- what htsjdk's CachingBAMFileIndex hands LinearBAMIndex."""
    if bai[:4] != b"BAI\1":
        raise ValueError("Invalid file header in BAM index")
    (n,) = struct.unpack_from("<i", bai, 4)
    p = 8
    out = []
    for _ in range(n):
        (nb,) = struct.unpack_from("<i", bai, p)
        p += 4
        for _ in range(nb):
            _, nc = struct.unpack_from("<Ii", bai, p)
            p += 8 + 16 * nc
        (ni,) = struct.unpack_from("<i", bai, p)
        p += 4
        e = list(struct.unpack_from(f"<{ni}Q", bai, p)) if ni else []
        p += 8 * ni
        out.append(e if nb > 0 else [])
    return out


def add_bai_splits(splits, dict_size, lin, first_voff, guess):
    """splits = [(start, length)] of one file in order; lin = linear_index();
    guess(beg, end) = BAMSplitGuesser.guessNextBAMRecordStart.  Returns
    [(vStart, vEnd)].  Raises LookupError where the Java code would throw
    (no contig with linear entries; a guessed first split)."""
    out = []
    n = len(splits)
    splits_end = 0
    ctg = -1
    b = 0

    def lin_of(c):
        if c >= len(lin):
            raise LookupError("no linear index for contig %d" % c)
        return lin[c]

    while True:  # :353-357
        ctg += 1
        li = lin_of(ctg)
        ctg_bins = len(li)
        if ctg_bins != 0:
            break
    next_start = li[b]
    last_start = 0
    new_split = None
    last_guessed = False
    while splits_end < n:  # :363
        fs, fl = splits[splits_end]
        splits_end += 1
        if splits_end >= n:
            break
        f_end = (fs + fl) << 16
        last_start = next_start
        while next_start < f_end and ctg < dict_size:  # :380
            if b + 1 >= ctg_bins:
                while True:
                    ctg += 1
                    b = 0
                    if ctg >= dict_size:
                        break
                    li = lin_of(ctg)
                    ctg_bins = len(li)
                    if ctg_bins != 0:
                        break
            if ctg < dict_size and len(li) > b:
                next_start = li[b]
                b += 1
        if fs == 0:  # :409
            new_split = [first_voff, next_start - 1]
            out.append(new_split)
        else:
            if last_start != next_start:
                if last_guessed:
                    new_split[1] = last_start - 1
                    last_guessed = False
                new_split = [last_start, next_start - 1]
                out.append(new_split)
            else:
                aligned = guess(fs, fs + fl)
                if new_split is None:
                    raise LookupError("guessed split with no split before it")
                new_split[1] = aligned - 1
                last_start = aligned
                next_start = aligned
                new_split = [aligned, aligned + 1]
                last_guessed = True
                out.append(new_split)
        last_start = next_start
    if splits_end == n and n > 0:  # :447
        if last_guessed:
            new_split[1] = last_start - 1
        fs, fl = splits[splits_end - 1]
        out.append([last_start, (fs + fl) << 16])
    return [tuple(x) for x in out]


def file_splits(size, split_size):
    """FileInputFormat byte splits of one file (SPLIT_SLOP 1.1)."""
    out = []
    rem = size
    while rem / split_size > 1.1:
        out.append((size - rem, split_size))
        rem -= split_size
    if rem:
        out.append((size - rem, rem))
    return out
