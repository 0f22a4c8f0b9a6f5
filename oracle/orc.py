"""ctypes binding of the C oracle (oracle/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as the
thing measured or shipped.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liborc.so not built: run `make -C oracle`")
        L = C.CDLL(path)
        u64, i32, i64, u32 = C.c_uint64, C.c_int32, C.c_int64, C.c_uint32
        P = C.c_void_p
        L.orc_open.argtypes = [P, u64, C.c_int, C.c_int, C.POINTER(P)]
        L.orc_close.argtypes = [P]
        L.orc_error.argtypes = [P]
        L.orc_error.restype = C.c_char_p
        for n in ("orc_nblocks", "orc_data_len", "orc_header_end", "orc_first_record_voff"):
            getattr(L, n).argtypes = [P]
            getattr(L, n).restype = u64
        L.orc_voff_of.argtypes = [P, u64]
        L.orc_voff_of.restype = u64
        L.orc_blocks.argtypes = [P]
        L.orc_blocks.restype = P
        L.orc_data.argtypes = [P]
        L.orc_data.restype = P
        L.orc_n_ref.argtypes = [P]
        L.orc_n_ref.restype = i32
        L.orc_l_text.argtypes = [P]
        L.orc_l_text.restype = i32
        L.orc_decode_span.argtypes = [P, u64, u64, P]
        L.orc_records_free.argtypes = [P]
        L.orc_splitting_index.argtypes = [P, u64, i32, C.POINTER(P), C.POINTER(u64)]
        L.orc_free.argtypes = [P]
        L.orc_murmurhash3.argtypes = [P, u64, i32]
        L.orc_murmurhash3.restype = i64
        L.orc_get_key.argtypes = [i32, i32, C.c_uint16, P, u32]
        L.orc_get_key.restype = i64
        L.orc_guess_record_start.argtypes = [P, P, u64, u64, u64, C.POINTER(u64)]
        L.orc_guess_record_start_hdr.argtypes = [P, P, u64, C.c_int32, u64, u64, C.POINTER(u64)]
        L.orc_guess_next_bgzf_block_start.argtypes = [P, u64, u64, u64]
        L.orc_guess_next_bgzf_block_start.restype = i64
        L.orc_get_splits.argtypes = [P, P, u64, P, P, u64, P, u64, P, P, C.POINTER(u64)]
        L.orc_bgzf_compress.argtypes = [P, u64, P, u64, C.c_int, C.c_int, P]
        L.orc_bgzf_compress.restype = u64
        L.orc_crc32.argtypes = [P, u64]
        L.orc_crc32.restype = u32
        L.orc_writable_encode.argtypes = [P, P, P, P]
        L.orc_writable_encode.restype = u64
        L.orc_writable_decode.argtypes = [P, u64, P, u64, P]
        L.orc_set_stringency.argtypes = [P, C.c_int]
        L.orc_scan.argtypes = [P, u64, C.c_int, C.c_int, C.c_int, i32, u64, C.POINTER(P), C.POINTER(u64), P]
        L.orc_scan_records.argtypes = [P, u64, C.c_int, C.c_int, u64, P, P, P]
        L.orc_record_invalid.argtypes = [P, i32, i32, P, C.c_int]
        L.orc_record_invalid.restype = C.c_int
        _LIB = L
    return _LIB


BLOCK_DTYPE = np.dtype([("coff", "<u8"), ("csize", "<u4"), ("isize", "<u4"),
                        ("crc", "<u4"), ("pad", "<u4"), ("ustart", "<u8")])

RECORD_FIELDS = [
    ("ref_id", np.int32), ("pos", np.int32), ("l_seq", np.int32), ("next_ref_id", np.int32),
    ("next_pos", np.int32), ("tlen", np.int32), ("l_read_name", np.uint8), ("mapq", np.uint8),
    ("bin", np.uint16), ("n_cigar", np.uint16), ("flag", np.uint16), ("key", np.int64),
    ("voff", np.uint64), ("offset", np.uint64), ("rest_len", np.uint32),
]


class _Records(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(name, C.c_void_p) for name, _ in RECORD_FIELDS]


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code


STRICT, LENIENT, SILENT = 0, 1, 2  # [htsjdk] ValidationStringency


class Stream:
    """A whole BGZF file inflated by zlib + BAM header parse (the oracle).
    stringency: validation of decode_span (htsjdk's default STRICT)."""

    def __init__(self, data: bytes, check_crc=False, parse_header=True, stringency=STRICT):
        L = lib()
        self._buf = C.create_string_buffer(bytes(data), len(data))
        self.file = bytes(data)
        self._h = C.c_void_p()
        rc = L.orc_open(self._buf, len(data), int(check_crc), int(parse_header), C.byref(self._h))
        if rc != 0:
            msg = L.orc_error(self._h).decode()
            L.orc_close(self._h)
            self._h = None
            raise OracleError(rc, msg)
        L.orc_set_stringency(self._h, stringency)

    def set_stringency(self, stringency):
        lib().orc_set_stringency(self._h, stringency)

    def close(self):
        if self._h:
            lib().orc_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def blocks(self):
        L = lib()
        n = L.orc_nblocks(self._h)
        if n == 0:
            return np.zeros(0, BLOCK_DTYPE)
        raw = C.string_at(L.orc_blocks(self._h), n * BLOCK_DTYPE.itemsize)
        return np.frombuffer(raw, BLOCK_DTYPE).copy()

    @property
    def data(self) -> bytes:
        L = lib()
        n = L.orc_data_len(self._h)
        return C.string_at(L.orc_data(self._h), n) if n else b""

    def data_array(self):
        """The inflated stream as a uint8 array over the oracle's buffer (no
        copy; valid while the Stream lives; any size, string_at stops at 2 GiB)."""
        L = lib()
        n = L.orc_data_len(self._h)
        if not n:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((C.c_uint8 * n).from_address(L.orc_data(self._h)))

    @property
    def data_len(self):
        return lib().orc_data_len(self._h)

    @property
    def n_ref(self):
        return lib().orc_n_ref(self._h)

    @property
    def header_end(self):
        return lib().orc_header_end(self._h)

    @property
    def first_record_voff(self):
        return lib().orc_first_record_voff(self._h)

    def voff_of(self, pos):
        return lib().orc_voff_of(self._h, pos)

    def decode_span(self, vstart, vend):
        """Returns (status, dict of numpy columns)."""
        L = lib()
        r = _Records()
        rc = L.orc_decode_span(self._h, vstart, vend, C.byref(r))
        out = _columns(r)
        L.orc_records_free(C.byref(r))
        return rc, out

    def writable_encode_span(self, vstart, vend):
        """SAMRecordWritable.write of every record of the span:
        (status, concatenated bytes, offsets[n+1])."""
        L = lib()
        r = _Records()
        rc = L.orc_decode_span(self._h, vstart, vend, C.byref(r))
        try:
            total = L.orc_writable_encode(L.orc_data(self._h), C.byref(r), None, None)
            out = C.create_string_buffer(max(total, 1))
            offs = np.zeros(r.n + 1, np.uint64)
            L.orc_writable_encode(L.orc_data(self._h), C.byref(r), out, offs.ctypes.data)
            return rc, out.raw[:total], offs
        finally:
            L.orc_records_free(C.byref(r))

    def decode_all(self):
        return self.decode_span(self.first_record_voff, (1 << 64) - 1)

    def splitting_index(self, granularity):
        L = lib()
        p = C.c_void_p()
        n = C.c_uint64()
        rc = L.orc_splitting_index(self._h, len(self.file), granularity, C.byref(p), C.byref(n))
        if rc != 0:
            raise OracleError(rc, L.orc_error(self._h).decode())
        b = C.string_at(p, n.value)
        L.orc_free(p)
        return b

    def guess_record_start(self, beg, end, header_n_ref=None):
        L = lib()
        out = C.c_uint64()
        if header_n_ref is None:
            rc = L.orc_guess_record_start(self._h, self._buf, len(self.file), beg, end, C.byref(out))
        else:
            rc = L.orc_guess_record_start_hdr(self._h, self._buf, len(self.file), header_n_ref, beg, end,
                                              C.byref(out))
        if rc != 0:
            raise OracleError(rc, L.orc_error(self._h).decode())
        return out.value

    def get_splits(self, starts, lengths, sbi=None):
        L = lib()
        n = len(starts)
        s = (C.c_uint64 * n)(*starts)
        ln = (C.c_uint64 * n)(*lengths)
        vs = (C.c_uint64 * max(n, 1))()
        ve = (C.c_uint64 * max(n, 1))()
        nout = C.c_uint64()
        sbuf = C.create_string_buffer(sbi, len(sbi)) if sbi is not None else None
        rc = L.orc_get_splits(self._h, self._buf, len(self.file), s, ln, n, sbuf,
                              len(sbi) if sbi is not None else 0, vs, ve, C.byref(nout))
        if rc != 0:
            raise OracleError(rc, L.orc_error(self._h).decode())
        return [(vs[i], ve[i]) for i in range(nout.value)]


def _columns(r):
    out = {}
    for name, dt in RECORD_FIELDS:
        p = getattr(r, name)
        if r.n and p:
            out[name] = np.frombuffer(C.string_at(p, r.n * np.dtype(dt).itemsize), dt).copy()
        else:
            out[name] = np.zeros(0, dt)
    return out


def writable_decode(buf: bytes, offs):
    """SAMRecordWritable.readFields per framed value: (status, columns)."""
    L = lib()
    offs = np.ascontiguousarray(offs, np.uint64)
    b = C.create_string_buffer(bytes(buf), max(len(buf), 1))
    r = _Records()
    rc = L.orc_writable_decode(b, len(buf), offs.ctypes.data, len(offs), C.byref(r))
    out = _columns(r)
    L.orc_records_free(C.byref(r))
    return rc, out


def murmurhash3(data: bytes, seed=0):
    return lib().orc_murmurhash3(C.c_char_p(bytes(data)), len(data), seed)


def get_key(ref_id, pos0, flag, var: bytes):
    return lib().orc_get_key(ref_id, pos0, flag, C.c_char_p(bytes(var)), len(var))


def guess_next_bgzf_block_start(file: bytes, beg, end):
    buf = C.create_string_buffer(file, len(file))
    return lib().orc_guess_next_bgzf_block_start(buf, len(file), beg, end)


def crc32(b: bytes):
    return lib().orc_crc32(C.c_char_p(bytes(b)), len(b))


def bgzf_compress(data: bytes, block_lens, level=5, eof=True) -> bytes:
    """[htsjdk] BlockCompressedOutputStream over `data` cut into block_lens
    (zlib raw deflater reset per block; see orc_bgzf_compress)."""
    L = lib()
    lens = np.ascontiguousarray(np.asarray(block_lens, dtype=np.uint32))
    assert int(lens.sum()) == len(data)
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = len(data) + 64 * len(lens) + 28 + 16  # stored sub-blocks: <= 5 x 5 B + 26 B framing per block
    out = np.empty(cap, dtype=np.uint8)
    n = L.orc_bgzf_compress(buf.ctypes.data, len(data), lens.ctypes.data if len(lens) else None, len(lens),
                            level, 1 if eof else 0, out.ctypes.data)
    if n == (1 << 64) - 1:
        raise OracleError(4, "zlib deflate failed")
    return out[:n].tobytes()


def record_invalid(rec: bytes, n_ref, ref_len=None, strict=True):
    """[htsjdk] SAMRecord.isValid restated (orc_record_invalid); rec starts at
    block_size."""
    import struct
    bs = struct.unpack_from("<i", rec, 0)[0]
    buf = C.create_string_buffer(bytes(rec), max(len(rec), 1))
    rl = None
    if ref_len is not None:
        arr = np.ascontiguousarray(ref_len, np.int32)
        rl = arr.ctypes.data
    return bool(lib().orc_record_invalid(buf, bs, n_ref, rl, 1 if strict else 0))


class _ScanResult(C.Structure):
    _fields_ = [("records", C.c_uint64), ("key_xor", C.c_uint64), ("voff_sum", C.c_uint64),
                ("blocks", C.c_uint64), ("u_bytes", C.c_uint64), ("status", C.c_int32), ("rewalks", C.c_int32),
                ("key_digest", C.c_uint64), ("voff_digest", C.c_uint64), ("field_digest", C.c_uint64 * 11),
                ("rest_crc", C.c_uint32), ("pad", C.c_uint32), ("rest_bytes", C.c_uint64)]
    FIELDS = ("ref_id", "pos", "l_read_name", "mapq", "bin", "n_cigar", "flag", "l_seq", "next_ref_id", "next_pos",
              "tlen")


DIGEST_P = 0x100000001B3  # ORC_DIGEST_P (hbam_oracle.h)
M64 = (1 << 64) - 1


def dmix(k):
    """MurmurHash3 fmix64 (the digest's per-record mix)."""
    k &= M64
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def digest(values):
    """Order-sensitive digest of a sequence of u64 (orc_scan_result.key_digest):
    sum_i dmix(x_i) * P^(n-1-i) mod 2^64, by Horner (small inputs / tests)."""
    d = 0
    for v in values:
        d = (d * DIGEST_P + dmix(int(v))) & M64
    return d


def digest_np(values):
    """digest() of a numpy integer column (signed columns sign-extended to
    64 bits, as orc_scan_result.field_digest), vectorized: (n, digest)."""
    x = np.asarray(values)
    x = (x.astype(np.int64) if x.dtype.kind == "i" else x.astype(np.uint64)).view(np.uint64)
    n = len(x)
    if n == 0:
        return 0, 0
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xFF51AFD7ED558CCD)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xC4CEB9FE1A85EC53)
        x = x ^ (x >> np.uint64(33))
        pw = np.empty(n, np.uint64)
        pw[0] = 1
        if n > 1:
            pw[1:] = np.cumprod(np.full(n - 1, DIGEST_P, np.uint64))
        return n, int((x * pw[::-1]).sum(dtype=np.uint64))


def digest_concat(parts):
    """Compose [(n, digest)] of consecutive record runs: D(A ++ B) = D(A) * P^|B| + D(B)."""
    d, n = 0, 0
    for k, dk in parts:
        d = (d * pow(DIGEST_P, int(k), 1 << 64) + int(dk)) & M64
        n += int(k)
    return n, d


def scan(data, threads=1, mode="decode", stringency=STRICT, granularity=4096, max_blocks=0):
    """orc_scan: the restated reader (mode 'decode') or indexer (mode 'index')
    over a whole file on `threads` host threads; data = bytes or a uint8
    ndarray.  Returns (result dict, .splitting-bai bytes or None)."""
    L = lib()
    if isinstance(data, np.ndarray):
        ptr, n = data.ctypes.data, data.nbytes
    else:
        keep = C.create_string_buffer(bytes(data), max(len(data), 1))
        ptr, n = C.addressof(keep), len(data)
    r = _ScanResult()
    out = C.c_void_p()
    olen = C.c_uint64()
    m = 0 if mode == "decode" else 1
    rc = L.orc_scan(ptr, n, threads, m, stringency, granularity, max_blocks,
                    C.byref(out) if m else None, C.byref(olen) if m else None, C.byref(r))
    sbi = None
    if m and out.value:
        sbi = C.string_at(out, olen.value)
        L.orc_free(out)
    d = {f: getattr(r, f) for f, _ in _ScanResult._fields_}
    d["field_digest"] = dict(zip(_ScanResult.FIELDS, list(r.field_digest)))
    d["rc"] = rc
    return d, sbi


def scan_records(data, cap, threads=1, stringency=STRICT):
    """orc_scan_records: the restated reader over a whole file on `threads`
    host threads, returning (result dict, keys int64[n], voffs uint64[n])."""
    L = lib()
    ptr, n = data.ctypes.data, data.nbytes
    keys = np.empty(max(cap, 1), np.int64)
    voffs = np.empty(max(cap, 1), np.uint64)
    r = _ScanResult()
    rc = L.orc_scan_records(ptr, n, threads, stringency, cap, keys.ctypes.data, voffs.ctypes.data, C.byref(r))
    d = {f: getattr(r, f) for f, _ in _ScanResult._fields_}
    d["field_digest"] = dict(zip(_ScanResult.FIELDS, list(r.field_digest)))
    d["rc"] = rc
    k = int(r.records)
    return d, keys[:k], voffs[:k]
