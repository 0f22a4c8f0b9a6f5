"""Independent pure-Python restatement of the key path (TEST INFRASTRUCTURE ONLY).

Written separately from oracle/hbam_oracle.c so that the two restatements can
cross-check each other on test.bam (no reference golden exists
for keys).  Pure-Python loops: small inputs only.

  murmurhash3  <- util/MurmurHash3.java:32-102 (quirk at :59), fmix :173-180
  get_key      <- BAMRecordReader.java:81-121
  records      <- [htsjdk] BAMRecordCodec.decode chain from the header end
  splitting_index <- SplittingBAMIndexer.java:248-290
  writable_encode <- SAMRecordWritable.java:55-64 ([htsjdk] BAMRecordCodec.encode)
"""
import struct
import zlib

M64 = (1 << 64) - 1


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def _signed64(x):
    return x - (1 << 64) if x >> 63 else x


def _signed32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def murmurhash3(key: bytes, seed: int = 0) -> int:
    """Java long returned by MurmurHash3.murmurhash3(byte[], int)."""
    c1, c2 = 0x87C37B91114253D5, 0x4CF5AD432745937F
    h1 = h2 = seed & M64
    n = len(key)
    nb = n // 16
    for i in range(nb):
        k1, k2 = struct.unpack_from("<QQ", key, 16 * i)
        k1 = (k1 * c1) & M64
        k1 = _rotl(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
        h1 = _rotl(h1, 27)
        h1 = (h1 + h2) & M64
        h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (k2 * c2) & M64
        k2 = _rotl(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
        h2 = ((h2 << 31) | (h1 >> 33)) & M64  # the :59 quirk
        h2 = (h2 + h1) & M64
        h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = key[16 * nb:]
    r = n & 15
    k1 = k2 = 0
    if r > 8:
        for j in range(8, r):
            k2 ^= tail[j] << (8 * (j - 8))
        k2 = (k2 * c2) & M64
        k2 = _rotl(k2, 33)
        k2 = (k2 * c1) & M64
        h2 ^= k2
    if r > 0:
        for j in range(0, min(r, 8)):
            k1 ^= tail[j] << (8 * j)
        k1 = (k1 * c1) & M64
        k1 = _rotl(k1, 31)
        k1 = (k1 * c2) & M64
        h1 ^= k1
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1 = _fmix(h1)
    h2 = _fmix(h2)
    h1 = (h1 + h2) & M64
    return _signed64(h1)


def get_key(ref_id, pos0, flag, var: bytes) -> int:
    start = _signed32(pos0 + 1)
    if not ((flag & 4) or ref_id < 0 or start < 0):
        return _signed64(((ref_id << 32) & M64) | (_signed32(start - 1) & M64))
    h = _signed32(murmurhash3(var, 0))
    return _signed64(((0x7FFFFFFF << 32) | (h & M64)) & M64)


def blocks(data: bytes):
    """[(coff, csize, isize)] by walking BSIZE (no framing checks beyond magic)."""
    out, p = [], 0
    while p < len(data):
        assert data[p:p + 4] == b"\x1f\x8b\x08\x04", p
        bsize = struct.unpack_from("<H", data, p + 16)[0] + 1
        isize = struct.unpack_from("<I", data, p + bsize - 4)[0]
        out.append((p, bsize, isize))
        p += bsize
    return out


def inflate(data: bytes):
    bl = blocks(data)
    parts, ustart = [], []
    u = 0
    for coff, csize, isize in bl:
        raw = zlib.decompressobj(-15).decompress(data[coff + 18:coff + csize - 8])
        assert len(raw) == isize
        parts.append(raw)
        ustart.append(u)
        u += isize
    return bl, ustart, b"".join(parts)


def voff(bl, ustart, pos):
    for k, (coff, csize, isize) in enumerate(bl):
        if ustart[k] == pos:
            return coff << 16
        if ustart[k] < pos < ustart[k] + isize:
            return (coff << 16) | (pos - ustart[k])
    coff, csize, _ = bl[-1]
    return (coff + csize) << 16


def records(data: bytes):
    """[(voff, key)] for every record of a well-formed BAM (no empty mid blocks)."""
    bl, ustart, u = inflate(data)
    assert u[:4] == b"BAM\x01"
    l_text = struct.unpack_from("<i", u, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", u, p)[0]
    p += 4
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", u, p)[0]
        p += 4 + ln + 4
    out = []
    while len(u) - p >= 4:
        bs = struct.unpack_from("<i", u, p)[0]
        ref, pos0 = struct.unpack_from("<ii", u, p + 4)
        flag = struct.unpack_from("<H", u, p + 18)[0]
        out.append((voff(bl, ustart, p), get_key(ref, pos0, flag, u[p + 36:p + 4 + bs])))
        p += 4 + bs
    return out


def splitting_index(data: bytes, g: int) -> bytes:
    bl, ustart, u = inflate(data)
    l_text = struct.unpack_from("<i", u, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", u, p)[0]
    p += 4
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", u, p)[0]
        p += 4 + ln + 4
    ent = [voff(bl, ustart, p)]
    i = 0
    while p < len(u):
        ptr = voff(bl, ustart, p)
        bs = struct.unpack_from("<i", u, p)[0]
        p += 4
        i += 1
        if i == g:
            i = 0
            ent.append(ptr)
        if bs > 0:
            p += bs
    ent.append(len(data) << 16)
    return b"".join(struct.pack(">Q", v) for v in ent)


def writable_encode(data: bytes) -> bytes:
    """SAMRecordWritable.write of every record, concatenated: each record is
    re-serialized from its parsed fields the way [htsjdk] BAMRecordCodec.encode
    does (block_size recomputed from the field lengths + attribute bytes,
    indexBin 0 for refID < 0, rest written back verbatim)."""
    bl, ustart, u = inflate(data)
    l_text = struct.unpack_from("<i", u, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", u, p)[0]
    p += 4
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", u, p)[0]
        p += 4 + ln + 4
    out = []
    while len(u) - p >= 4:
        bs = struct.unpack_from("<i", u, p)[0]
        (ref, pos0, lrn, mapq, bin_, ncig, flag, lseq, nref, npos,
         tlen) = struct.unpack_from("<iiBBHHHiiii", u, p + 4)
        rest = u[p + 36:p + 4 + bs]
        var = lrn + 4 * ncig + (lseq + 1) // 2 + lseq
        attrs = len(rest) - var
        out.append(struct.pack("<iiiBBHHHiiii", 32 + var + attrs, ref, pos0, lrn, mapq,
                               bin_ if ref >= 0 else 0, ncig, flag, lseq, nref, npos, tlen))
        out.append(rest)
        p += 4 + bs
    return b"".join(out)


# ---------------------------------------------------------------------------
# [htsjdk] SAMRecord.isValid under ValidationStringency.STRICT, restated a
# second time (independently of orc_record_invalid) over a decoded record:
# the two restatements are cross-checked by tests/test_strict.py.  Rule list:
# DESIGN.md 2.1.  rec = bytes starting at block_size.
# ---------------------------------------------------------------------------
def _reg2bin(beg, end):
    end -= 1
    for shift, off in ((14, 4681), (17, 585), (20, 73), (23, 9), (26, 1)):
        if beg >> shift == end >> shift:
            return off + (beg >> shift)
    return 0


def _aux_tags(aux: bytes):
    """{tag: Z-string length or None}; None if the aux block does not parse."""
    tags, i = {}, 0
    sizes = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}
    while i + 3 <= len(aux):
        tag, ty = aux[i:i + 2].decode("latin-1"), chr(aux[i + 2])
        i += 3
        if ty in sizes:
            n, zl = sizes[ty], None
        elif ty in "ZH":
            j = aux.find(b"\0", i)
            j = len(aux) if j < 0 else j
            zl, n = j - i, j - i + 1
        elif ty == "B":
            if i + 5 > len(aux):
                return tags
            sub, cnt = chr(aux[i]), struct.unpack_from("<i", aux, i + 1)[0]
            if cnt < 0:
                return tags
            n, zl = 5 + cnt * (1 if sub in "cC" else 2 if sub in "sS" else 4), None
        else:
            return tags
        tags.setdefault(tag, zl)
        if n > len(aux) - i:
            return tags
        i += n
    return tags


def record_invalid(rec: bytes, n_ref: int, ref_len=None, strict=True) -> bool:
    (bs, ref, pos, lrn, mapq, bin_, ncig, flag, lseq, nref, npos, tlen) = struct.unpack_from("<iiiBBHHHiiii", rec, 0)
    if lrn < 1 or lseq < 0 or 32 + lrn + 4 * ncig + (lseq + 1) // 2 + lseq > bs:
        return True
    cig = [struct.unpack_from("<I", rec, 36 + lrn + 4 * k)[0] for k in range(ncig)]
    ops = [(c & 15, c >> 4) for c in cig]
    if any(op > 8 for op, _ in ops):
        return True
    if not strict:
        return False
    M, I, D, N, S, H, P, EQ, X = range(9)
    paired, unmapped = bool(flag & 1), bool(flag & 4)
    if not paired:
        if flag & (2 | 8 | 0x20 | 0x40 | 0x80) or nref != -1:
            return True
    else:
        if (nref == -1) != (npos == -1):
            return True
        if nref != -1 and ref_len is not None and npos + 1 > ref_len[nref]:
            return True
        if nref == -1 and not flag & 8:
            return True
        if not flag & 0xC0:
            return True
    if unmapped:
        if flag & 0x900 or mapq:
            return True
    elif not ncig or n_ref == 0:
        return True
    if (ref == -1) != (pos == -1):
        return True
    if ref != -1 and ref_len is not None and pos + 1 > ref_len[ref]:
        return True
    real = {M, I, D, N, EQ, X}
    if not unmapped:
        if any(ln == 0 for _, ln in ops) or not any(op in real for op, _ in ops):
            return True
        last = len(ops) - 1
        for k, (op, _) in enumerate(ops):
            if op == H and 0 < k < last:
                return True
            if op == S and 0 < k < last:
                ok = (k == 1 and (ops[0][0] == H or (len(ops) == 3 and ops[2][0] == H))) or \
                     (k == last - 1 and ops[last][0] == H)
                if not ok:
                    return True
            if op == P and k > 0 and (k == last or ops[k - 1][0] not in real or ops[k + 1][0] not in real):
                return True
        # two I (or two D) with no M/N/=/X or P between them
        seg = []
        for op, _ in ops + [(M, 1)]:
            if op in (M, N, EQ, X, P):
                if seg.count(I) > 1 or seg.count(D) > 1:
                    return True
                seg = []
            elif op in (I, D):
                seg.append(op)
        at = pos + 1
        for op, ln in ops:
            if op in (M, EQ, X) and ref >= 0 and ref_len is not None and at + ln - 1 > ref_len[ref]:
                return True
            if op in (M, D, N, EQ, X):
                at += ln
    rlen = sum(ln for op, ln in ops if op in (M, D, N, EQ, X))
    qlen = sum(ln for op, ln in ops if op in (M, I, S, EQ, X))
    end = 0 if unmapped else pos + rlen
    if end <= 0:
        end = pos + 1
    if _reg2bin(pos, end) != bin_:
        return True
    if lseq and ncig and qlen != lseq:
        return True
    if lseq == 0 and not flag & 0x100:
        tags = _aux_tags(rec[36 + lrn + 4 * ncig:4 + bs])
        if "FZ" not in tags and not (tags.get("CQ") and tags.get("CS")):
            return True
    return False
