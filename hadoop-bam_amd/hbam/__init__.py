"""ctypes binding of libhbam.so (include/hbam.h) for tests and bench.py.

There is no Python or CPU implementation of the hot path here: every call goes
through the C ABI into the gfx950 kernels.  If the library is missing this
module raises at import time (no silent fallback).
"""
import ctypes as C
import os
import re

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HBAM_LIB: load another in-tree build of the same ABI (scripts/probe_inflate.py compares variants)
LIB_PATH = os.environ.get("HBAM_LIB") or os.path.join(_PKG, "lib", "libhbam.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "hbam.h")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is not built: run `make -C hadoop-bam_amd` (libhbam has no CPU fallback)")

_L = C.CDLL(LIB_PATH)

OK, E_FORMAT, E_TRUNC, E_ARG, E_IO, E_DEVICE, E_STATE, E_NOMEM = range(8)
ERROR_NAMES = {1: "SAMFormatException", 2: "FileTruncatedException", 3: "IllegalArgumentException",
               4: "IOException", 5: "DeviceError", 6: "IllegalStateException", 7: "OutOfMemoryError"}

u64, i64, i32, u32, P = C.c_uint64, C.c_int64, C.c_int32, C.c_uint32, C.c_void_p


STRICT, LENIENT, SILENT = 0, 1, 2  # hadoopbam.samheaderreader.validation-stringency


class Opts(C.Structure):
    _fields_ = [("device", i32), ("check_crc", i32), ("stringency", i32), ("parallel_reads", i32),
                ("window_bytes", u64), ("batch_records", u64)]


def _opts(device=0, check_crc=False, stringency=STRICT, window_bytes=0, parallel_reads=False, batch_records=0):
    return Opts(device, int(check_crc), stringency, int(parallel_reads), window_bytes, batch_records)


class HeaderInfo(C.Structure):
    _fields_ = [("n_ref", i32), ("l_text", i32), ("first_record_voff", u64), ("file_size", u64),
                ("text", C.c_char_p)]


_COLS = [("ref_id", np.int32), ("pos", np.int32), ("l_seq", np.int32), ("next_ref_id", np.int32),
         ("next_pos", np.int32), ("tlen", np.int32), ("l_read_name", np.uint8), ("mapq", np.uint8),
         ("bin", np.uint16), ("n_cigar", np.uint16), ("flag", np.uint16), ("key", np.int64),
         ("voff", np.uint64), ("rest_off", np.uint64), ("rest_len", np.uint32)]


class Batch(C.Structure):
    _fields_ = [("n", u64)] + [(n, P) for n, _ in _COLS] + [("data", P), ("data_len", u64),
                                                            ("status", i32), ("reserved", i32),
                                                            ("next_voff", u64)]


class GpuStats(C.Structure):
    _fields_ = [("n_blocks", u64), ("compressed_bytes", u64), ("inflated_bytes", u64), ("records", u64),
                ("first_voff", u64), ("last_voff", u64), ("key_xor", u64), ("voff_sum", u64),
                ("ms_locate", C.c_float), ("ms_inflate", C.c_float), ("ms_huff", C.c_float),
                ("ms_lz77", C.c_float), ("ms_chain", C.c_float), ("ms_decode", C.c_float),
                ("ms_total", C.c_float), ("status", i32), ("link_fallbacks", i32),
                ("inflate_launches", i32), ("link_rewalks", i32), ("windows", i32), ("ms_tables", C.c_float),
                ("record_fallbacks", i32), ("key_digest", u64), ("voff_digest", u64)]


def _sig(name, res, args):
    f = getattr(_L, name)
    f.restype = res
    f.argtypes = args
    return f


_sig("hbam_abi_version", i32, [])
_sig("hbam_release_cached_memory", u64, [])
_sig("hbam_open", C.c_int, [C.c_char_p, C.POINTER(Opts), C.POINTER(P)])
_sig("hbam_open_mem", C.c_int, [P, u64, C.POINTER(Opts), C.POINTER(P)])
_sig("hbam_open_bgzf", C.c_int, [P, u64, C.POINTER(Opts), C.POINTER(P)])
# hbam_read_fn: int64 (*)(void *user, uint64 offset, void *dst, uint64 len)
READ_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64)
_sig("hbam_open_reader", C.c_int, [u64, READ_FN, P, C.POINTER(Opts), C.POINTER(P)])
_sig("hbam_close", None, [P])
_sig("hbam_last_error", C.c_char_p, [P])
_sig("hbam_free", None, [P])
_sig("hbam_header", C.c_int, [P, C.POINTER(HeaderInfo)])
_sig("hbam_ref", C.c_int, [P, i32, C.POINTER(C.c_char_p), C.POINTER(i32)])
_sig("hbam_decode_span", C.c_int, [P, u64, u64, u64, C.POINTER(Batch)])
_sig("hbam_decode_span_device", C.c_int, [P, u64, u64, i32, C.POINTER(GpuStats)])
_sig("hbam_reader_position", C.c_int, [P, u64, C.POINTER(u64)])
_sig("hbam_pipeline_counters", C.c_int, [P, C.POINTER(u64)])
_sig("hbam_inflate_token_count", C.c_int, [P, C.POINTER(u64)])
_sig("hbam_file_stats", C.c_int, [P, C.POINTER(u64), C.POINTER(u64)])
_sig("hbam_bytes_read", C.c_int, [P, C.POINTER(u64)])
_sig("hbam_prefetch", C.c_int, [P, u64, u64])
_sig("hbam_splitting_index_for_records", C.c_int, [C.POINTER(Opts), P, u64, i32, u64, C.POINTER(P), C.POINTER(u64)])
_sig("hbam_build_splitting_index", C.c_int, [P, i32, C.POINTER(P), C.POINTER(u64)])
_sig("hbam_splitting_entries", C.c_int, [P, u64, u64, i32, u64, C.POINTER(P), C.POINTER(u64), C.POINTER(u64)])
_sig("hbam_guess_record_starts", C.c_int, [P, P, P, u64, P])
_sig("hbam_guess_record_starts_hdr", C.c_int, [P, i32, P, P, u64, P])
_sig("hbam_guess_bgzf_block_starts", C.c_int, [P, P, P, u64, P])
_sig("hbam_get_splits", C.c_int, [P, P, P, u64, P, u64, P, P, C.POINTER(u64)])
_sig("hbam_get_splits_bai", C.c_int, [P, P, P, u64, P, u64, P, u64, P, P, C.POINTER(u64)])
_sig("hbam_blocks", C.c_int, [P, P, P, P, P, u64, C.POINTER(u64)])
_sig("hbam_read_inflated", C.c_int, [P, u64, u64, P])
_sig("hbam_get_key0", i64, [i32, i32])
_sig("hbam_get_key", i64, [i32, i32])
_sig("hbam_murmurhash3", i64, [P, u64, i32])
_sig("hbam_device_count", i32, [])
_sig("hbam_gpu_create", C.c_int, [i32, C.POINTER(P)])
_sig("hbam_gpu_destroy", None, [P])
_sig("hbam_gpu_error", C.c_char_p, [P])
_sig("hbam_gpu_load", C.c_int, [P, P, u64])
_sig("hbam_gpu_set_window", C.c_int, [P, u64])
_sig("hbam_gpu_index", C.c_int, [P, i32, C.POINTER(P), C.POINTER(u64), C.POINTER(C.c_float)])
_sig("hbam_gpu_run", C.c_int, [P, i32, C.POINTER(GpuStats)])
_sig("hbam_gpu_fetch", C.c_int, [P, P, P, u64])
_sig("hbam_encode_writables", C.c_int, [P, P, u64, P, C.POINTER(u64)])
_sig("hbam_decode_writables", C.c_int, [P, P, u64, P, u64, C.POINTER(Batch)])
_sig("hbam_open_codec", C.c_int, [C.POINTER(Opts), C.POINTER(P)])
_sig("hbam_gpu_encode_writables", C.c_int, [P, i32, C.POINTER(C.c_float), C.POINTER(u64)])
_sig("hbam_gpu_fetch_encoded", C.c_int, [P, u64, u64, P])
_sig("hbam_gpu_reload", C.c_int, [P, P, u64, i32, C.POINTER(C.c_float)])
_sig("hbam_gpu_run_streamed", C.c_int, [P, P, u64, u64, C.POINTER(GpuStats)])
_sig("hbam_host_alloc", P, [u64])
_sig("hbam_host_free", None, [P])
_sig("hbam_gpu_d2d_bandwidth", C.c_int, [P, u64, i32, C.POINTER(C.c_float)])
_sig("hbam_bgzf_compress", C.c_int, [C.POINTER(Opts), P, u64, P, u64, i32, i32, i32, C.POINTER(P), C.POINTER(u64)])
_sig("hbam_gpu_bgzf_compress", C.c_int, [P, i32, i32, i32, C.POINTER(C.c_float), C.POINTER(u64)])
_sig("hbam_gpu_fetch_compressed", C.c_int, [P, u64, u64, P])

BGZF_EOF = 1
HTSJDK_BLOCK_SIZE = 65498  # ISIZE of every full block of test.bam (htsjdk-written)


def lib():
    return _L


def exported_symbols_from_header(path=HEADER_PATH):
    """Function names declared in include/hbam.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hbam_[a-z0-9_]+)\s*\(", txt)))


class HbamError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def device_count():
    return _L.hbam_device_count()


def murmurhash3(data: bytes, seed=0):
    return _L.hbam_murmurhash3(C.c_char_p(bytes(data)), len(data), seed)


def bgzf_compress(data, block_lens=None, block_size=HTSJDK_BLOCK_SIZE, level=5, eof=True, device=0):
    """[htsjdk] BlockCompressedOutputStream over `data` on the GPU
    (hbam_bgzf_compress): the BGZF file bytes.  block_lens (optional) cuts
    the payload as the writer's flushes did; else every block_size bytes."""
    if isinstance(data, np.ndarray):
        buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        n = buf.nbytes
        ptr = buf.ctypes.data if n else None
    else:
        buf = C.create_string_buffer(bytes(data), max(len(data), 1))
        ptr, n = buf, len(data)
    lens_ptr, nl = None, 0
    if block_lens is not None:
        # an explicit list (even an empty one) is passed as a non-NULL pointer,
        # so the C side checks that it covers the payload
        lens = np.ascontiguousarray(np.asarray(block_lens, dtype=np.uint32))
        keep = lens if len(lens) else np.zeros(1, np.uint32)
        lens_ptr, nl = keep.ctypes.data, len(lens)
    o = _opts(device)
    out = P()
    olen = u64()
    rc = _L.hbam_bgzf_compress(C.byref(o), ptr, n, lens_ptr, nl, block_size, level,
                               BGZF_EOF if eof else 0, C.byref(out), C.byref(olen))
    if rc != OK:
        raise HbamError(rc, _L.hbam_gpu_error(None).decode())
    try:
        return C.string_at(out, olen.value)
    finally:
        _L.hbam_free(out)


def release_cached_memory():
    """hbam_release_cached_memory: the process-wide block caches back to HIP (bytes)."""
    return int(_L.hbam_release_cached_memory())


def get_key0(ref_idx, start0):
    return _L.hbam_get_key0(ref_idx, start0)


def get_key(ref_idx, alignment_start):
    return _L.hbam_get_key(ref_idx, alignment_start)


def splitting_index_for_records(voffs, granularity, file_size, device=0) -> bytes:
    """Write-time .splitting-bai (SplittingBAMIndexer.processAlignment over
    records with these voffs, then finish(file_size)), entries on the GPU."""
    v = np.ascontiguousarray(voffs, np.uint64)
    keep = v if len(v) else np.zeros(1, np.uint64)
    out = P()
    n = u64()
    rc = _L.hbam_splitting_index_for_records(C.byref(_opts(device)), keep.ctypes.data, len(v), granularity,
                                             file_size, C.byref(out), C.byref(n))
    if rc != OK:
        raise HbamError(rc, _L.hbam_last_error(None).decode())
    try:
        return C.string_at(out, n.value)
    finally:
        _L.hbam_free(out)


def _stats_dict(st):
    return {f: getattr(st, f) for f, _ in GpuStats._fields_}


def _batch_dict(b, rc):
    out = {"status": rc, "next_voff": b.next_voff}
    for name, dt in _COLS:
        p = getattr(b, name)
        nb = b.n * np.dtype(dt).itemsize
        out[name] = np.frombuffer(C.string_at(p, nb), dt).copy() if b.n else np.zeros(0, dt)
    out["data"] = C.string_at(b.data, b.data_len) if b.data_len else b""
    return out


def _decode_writables(h, buf, offs, raise_on_error):
    offs = np.ascontiguousarray(offs, np.uint64)
    keep = C.create_string_buffer(bytes(buf), max(len(buf), 1))
    b = Batch()
    rc = _L.hbam_decode_writables(h, keep, len(buf), offs.ctypes.data, len(offs), C.byref(b))
    if rc != OK and (raise_on_error or rc not in (E_FORMAT, E_TRUNC, E_ARG)):
        raise HbamError(rc, _L.hbam_last_error(h).decode(errors="replace"))
    return _batch_dict(b, rc)


class PinnedBuffer:
    """Page-locked host memory from hbam_host_alloc, as a numpy uint8 view."""

    def __init__(self, nbytes):
        self.ptr = _L.hbam_host_alloc(nbytes)
        if not self.ptr:
            raise HbamError(E_NOMEM, "hbam_host_alloc failed")
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]

    def close(self):
        if self.ptr:
            self.array = None
            _L.hbam_host_free(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Codec:
    """SAMRecordWritable.readFields in bulk on a GPU with no file open
    (a reducer's view: hbam_open_codec + hbam_decode_writables)."""

    def __init__(self, device=0):
        self._h = P()
        rc = _L.hbam_open_codec(C.byref(_opts(device)), C.byref(self._h))
        if rc != OK:
            msg = _L.hbam_last_error(self._h).decode(errors="replace")
            _L.hbam_close(self._h)
            self._h = None
            raise HbamError(rc, msg)

    def decode_writables(self, buf: bytes, offs, raise_on_error=True):
        return _decode_writables(self._h, buf, offs, raise_on_error)

    def close(self):
        if self._h:
            _L.hbam_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def reader_callback(read):
    """hbam_read_fn over a Python positioned read: read(offset, n) -> bytes
    (fewer than n only at the end of the file); an exception, or more than n
    bytes (which would overrun the library's page-locked buffer), is an I/O
    error (-1).  Keep the returned object alive as long as the ctx."""
    def cb(user, off, dst, n):
        try:
            b = read(int(off), int(n))
        except Exception:
            return -1
        if b is None or len(b) > n:
            return -1
        if b:
            C.memmove(dst, b, len(b))
        return len(b)
    return READ_FN(cb)


class BamFile:
    """An opened BAM (or plain BGZF with bam=False) on one GPU.  path= opens
    a file split-locally (only the windows a decode needs are read, with
    pread); reader= + size= reads through a positioned-read callback
    (hbam_open_reader: read(offset, n) -> bytes, as a Hadoop FSDataInputStream
    does through JNI; parallel_reads: it may be called from several library
    threads at once); window_bytes = compressed bytes per HBM window (0: 4 GiB);
    batch_records = the max_records decode_span / scan_batches will use (the
    batch slots are then page-locked from the open on, hbam_opts)."""

    def __init__(self, data: bytes = None, path: str = None, device=0, bam=True, check_crc=False,
                 stringency=STRICT, window_bytes=0, reader=None, size=None, parallel_reads=False,
                 batch_records=0):
        self._h = P()
        o = _opts(device, check_crc, stringency, window_bytes, parallel_reads, batch_records)
        if reader is not None:
            if size is None:
                raise ValueError("BamFile(reader=...) needs size= (the file length)")
            self._cb = reader_callback(reader)
            rc = _L.hbam_open_reader(size, self._cb, None, C.byref(o), C.byref(self._h))
            self.size = size
        elif path is not None:
            rc = _L.hbam_open(path.encode(), C.byref(o), C.byref(self._h))
            self.size = os.path.getsize(path)
        else:
            self._buf = C.create_string_buffer(bytes(data), len(data))
            fn = _L.hbam_open_mem if bam else _L.hbam_open_bgzf
            rc = fn(self._buf, len(data), C.byref(o), C.byref(self._h))
            self.size = len(data)
        if rc != OK:
            msg = _L.hbam_last_error(self._h).decode(errors="replace")
            _L.hbam_close(self._h)
            self._h = None
            raise HbamError(rc, msg)
        self.bam = bam
        self._last_n = 0

    def close(self):
        if self._h:
            _L.hbam_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, rc):
        return HbamError(rc, _L.hbam_last_error(self._h).decode(errors="replace"))

    def header(self):
        h = HeaderInfo()
        rc = _L.hbam_header(self._h, C.byref(h))
        if rc != OK:
            raise self._err(rc)
        text = C.string_at(h.text, h.l_text).decode(errors="replace") if h.l_text else ""
        return {"n_ref": h.n_ref, "l_text": h.l_text, "first_record_voff": h.first_record_voff,
                "file_size": h.file_size, "text": text}

    def file_stats(self):
        """(BGZF blocks, inflated bytes) of the whole file."""
        nb, us = u64(), u64()
        rc = _L.hbam_file_stats(self._h, C.byref(nb), C.byref(us))
        if rc != OK:
            raise self._err(rc)
        return nb.value, us.value

    def bytes_read(self):
        """Host -> HBM bytes this file has copied so far."""
        n = u64()
        rc = _L.hbam_bytes_read(self._h, C.byref(n))
        if rc != OK:
            raise self._err(rc)
        return n.value

    def prefetch(self, lo, hi):
        rc = _L.hbam_prefetch(self._h, lo, hi)
        if rc != OK:
            raise self._err(rc)

    def reader_position(self, i):
        """BAMRecordReader.getProgress's in.position() after record i of the last batch."""
        v = u64()
        rc = _L.hbam_reader_position(self._h, i, C.byref(v))
        if rc != OK:
            raise self._err(rc)
        return v.value

    def pipeline_counters(self):
        """Cumulative path counters of the ctx (hbam_pipeline_counters)."""
        v = (u64 * 5)()
        rc = _L.hbam_pipeline_counters(self._h, v)
        if rc != OK:
            raise self._err(rc)
        return dict(zip(("link_fallbacks", "link_rewalks", "record_fallbacks", "inflate_launches",
                         "records_after_stop"),
                        (int(x) for x in v)))

    def inflate_token_count(self):
        """LZ77 tokens phase A wrote in the last pass over the current window
        (hbam_inflate_token_count)."""
        v = u64()
        rc = _L.hbam_inflate_token_count(self._h, C.byref(v))
        if rc != OK:
            raise self._err(rc)
        return int(v.value)

    def decode_span_device(self, vstart, vend, timing=False, decode=True, digest=True):
        """The span decoded with the records left in HBM: stats dict."""
        st = GpuStats()
        flags = (1 if timing else 0) | (0 if decode else 2) | (4 if digest else 0)
        rc = _L.hbam_decode_span_device(self._h, vstart, vend, flags, C.byref(st))
        if rc != OK:
            raise self._err(rc)
        return _stats_dict(st)

    def ref(self, i):
        name = C.c_char_p()
        ln = i32()
        rc = _L.hbam_ref(self._h, i, C.byref(name), C.byref(ln))
        if rc != OK:
            raise self._err(rc)
        return name.value.decode(), ln.value

    def decode_span(self, vstart, vend, raise_on_error=True, max_records=0):
        """SoA dict for FileVirtualSplit [vstart, vend) (at most max_records
        records; 0 = all); 'status' holds the status of a record that ended
        the span early, 'next_voff' where the next batch continues."""
        b = Batch()
        rc = _L.hbam_decode_span(self._h, vstart, vend, max_records, C.byref(b))
        if rc != OK and (raise_on_error or b.n == 0 and rc not in (E_FORMAT, E_TRUNC, E_ARG, E_IO)):
            raise self._err(rc)
        self._last_n = b.n
        return _batch_dict(b, rc)

    def iter_batches(self, vstart, vend, max_records, raise_on_error=True):
        """The split in bounded batches (BAMRecordReader's iteration)."""
        v = vstart
        while v < vend:
            r = self.decode_span(v, vend, raise_on_error=raise_on_error, max_records=max_records)
            if len(r["key"]):
                yield r
            if r["status"] != OK or not len(r["key"]):
                if r["status"] != OK:
                    yield r
                return
            v = r["next_voff"]

    def scan_batches(self, vstart, vend, max_records):
        """The split through hbam_decode_span in bounded batches, as a JNI
        caller iterates it, leaving each batch in the library's pinned host
        columns (no Python copies): (records, batches, rest bytes)."""
        b = Batch()
        v, n, k, nbytes = vstart, 0, 0, 0
        while v < vend:
            rc = _L.hbam_decode_span(self._h, v, vend, max_records, C.byref(b))
            if rc != OK:
                raise self._err(rc)
            if b.n == 0:
                break
            n += b.n
            k += 1
            nbytes += b.data_len
            v = b.next_voff
        self._last_n = b.n
        return n, k, nbytes

    def encode_writables(self):
        """SAMRecordWritable.write of every record of the last decode_span
        (GPU): (bytes, offsets[n+1])."""
        n = u64()
        rc = _L.hbam_encode_writables(self._h, None, 0, None, C.byref(n))
        if rc != OK:
            raise self._err(rc)
        total = n.value
        out = C.create_string_buffer(max(total, 1))
        offs = np.zeros(self._last_n + 1, np.uint64)
        rc = _L.hbam_encode_writables(self._h, out, total, offs.ctypes.data, C.byref(n))
        if rc != OK:
            raise self._err(rc)
        return out.raw[:total], offs

    def decode_writables(self, buf: bytes, offs, raise_on_error=True):
        return _decode_writables(self._h, buf, offs, raise_on_error)

    def decode_all(self, raise_on_error=True):
        return self.decode_span(self.header()["first_record_voff"], (1 << 64) - 1, raise_on_error)

    def splitting_index(self, granularity=4096) -> bytes:
        p = P()
        n = u64()
        rc = _L.hbam_build_splitting_index(self._h, granularity, C.byref(p), C.byref(n))
        if rc != OK:
            raise self._err(rc)
        b = C.string_at(p, n.value)
        _L.hbam_free(p)
        return b

    def splitting_entries(self, vstart, vend, granularity, ordinal0):
        """This split's part of SplittingBAMIndexer.index (hbam_splitting_entries):
        (records of the split, [voffs of the records at global ordinals k*g - 1])."""
        p = P()
        ne = u64()
        nr = u64()
        rc = _L.hbam_splitting_entries(self._h, vstart, vend, granularity, ordinal0, C.byref(p), C.byref(ne),
                                       C.byref(nr))
        if rc != OK:
            raise self._err(rc)
        try:
            ent = np.frombuffer(C.string_at(p, 8 * ne.value), np.uint64).copy() if ne.value else np.zeros(0, np.uint64)
        finally:
            _L.hbam_free(p)
        return nr.value, ent

    def guess_record_starts(self, begs, ends, header_n_ref=None):
        """BAMSplitGuesser.guessNextBAMRecordStart for many split points;
        header_n_ref: the sequence count of a header read from another stream
        (the three-argument constructor), None = the file's own header."""
        n = len(begs)
        b = np.ascontiguousarray(begs, np.uint64)
        e = np.ascontiguousarray(ends, np.uint64)
        out = np.zeros(max(n, 1), np.uint64)
        if header_n_ref is None:
            rc = _L.hbam_guess_record_starts(self._h, b.ctypes.data, e.ctypes.data, n, out.ctypes.data)
        else:
            rc = _L.hbam_guess_record_starts_hdr(self._h, int(header_n_ref), b.ctypes.data, e.ctypes.data, n,
                                                 out.ctypes.data)
        if rc != OK:
            raise self._err(rc)
        return [int(x) for x in out[:n]]

    def guess_bgzf_block_starts(self, begs, ends):
        """BGZFSplitGuesser.guessNextBGZFBlockStart for many split points."""
        n = len(begs)
        b = np.ascontiguousarray(begs, np.uint64)
        e = np.ascontiguousarray(ends, np.uint64)
        out = np.zeros(max(n, 1), np.uint64)
        rc = _L.hbam_guess_bgzf_block_starts(self._h, b.ctypes.data, e.ctypes.data, n, out.ctypes.data)
        if rc != OK:
            raise self._err(rc)
        return [int(x) for x in out[:n]]

    def get_splits(self, starts, lengths, sbi: bytes = None, bai: bytes = None):
        """BAMInputFormat.getSplits for one file's FileSplits: from the
        .splitting-bai (sbi), else -- with bai given, the BAI split
        calculator enabled -- from the .bai's linear index, else
        probabilistic.  [(vStart, vEnd)]."""
        n = len(starts)
        s = np.ascontiguousarray(starts, np.uint64)
        ln = np.ascontiguousarray(lengths, np.uint64)
        vs = np.zeros(max(n, 1), np.uint64)
        ve = np.zeros(max(n, 1), np.uint64)
        nout = u64()
        sb = C.create_string_buffer(sbi, len(sbi)) if sbi is not None else None
        bb = C.create_string_buffer(bai, len(bai)) if bai is not None else None
        rc = _L.hbam_get_splits_bai(self._h, s.ctypes.data, ln.ctypes.data, n, sb,
                                    len(sbi) if sbi is not None else 0, bb, len(bai) if bai is not None else 0,
                                    vs.ctypes.data, ve.ctypes.data, C.byref(nout))
        if rc != OK:
            raise self._err(rc)
        return [(int(vs[i]), int(ve[i])) for i in range(nout.value)]

    def blocks(self):
        n = u64()
        _L.hbam_blocks(self._h, None, None, None, None, 0, C.byref(n))
        k = n.value
        coff = np.zeros(max(k, 1), np.uint64)
        csize = np.zeros(max(k, 1), np.uint32)
        isize = np.zeros(max(k, 1), np.uint32)
        ustart = np.zeros(max(k, 1), np.uint64)
        rc = _L.hbam_blocks(self._h, coff.ctypes.data, csize.ctypes.data, isize.ctypes.data,
                            ustart.ctypes.data, k, C.byref(n))
        if rc != OK:
            raise self._err(rc)
        return {"coff": coff[:k], "csize": csize[:k], "isize": isize[:k], "ustart": ustart[:k]}

    def read_inflated(self, pos, length):
        buf = C.create_string_buffer(max(length, 1))
        rc = _L.hbam_read_inflated(self._h, pos, length, buf)
        if rc != OK:
            raise self._err(rc)
        return buf.raw[:length]


class BAMSplitGuesser:
    """BAMSplitGuesser (BAMSplitGuesser.java:80-235) over a seekable stream,
    as java/.../GpuBAMSplitGuesser.java: the stream is read through
    hbam_open_reader by positioned reads (seek + read under a lock, one at a
    time), so only the bytes a guess needs are read; the BGZF block search,
    inflate and record checks run on the GPU (hbam_guess.hip).
      BAMSplitGuesser(ss)                  the two-argument constructor: the
                                           header comes from ss, whose first
                                           four bytes must be the BGZF magic
      BAMSplitGuesser(ss, header_stream)   the three-argument one: refIDs are
                                           bounded by header_stream's sequence
                                           dictionary (a seekable BAM stream)
    ss / header_stream: binary file objects with seek / read."""

    BGZF_MAGIC = b"\x1f\x8b\x08\x04"

    def __init__(self, ss, header_stream=None, device=0):
        import threading
        lock = threading.Lock()

        def positioned(stream):
            def read(off, n):
                with lock:
                    stream.seek(off)
                    return stream.read(n)
            return read

        def size_of(stream):
            with lock:
                return stream.seek(0, os.SEEK_END)

        self._n_ref = None
        if header_stream is not None and header_stream is not ss:
            with BamFile(reader=positioned(header_stream), size=size_of(header_stream), device=device,
                         stringency=SILENT) as hf:
                self._n_ref = hf.header()["n_ref"]
        self._f = BamFile(reader=positioned(ss), size=size_of(ss), device=device, stringency=SILENT)
        if header_stream is None:  # :86-90 the secondary magic check
            with lock:
                ss.seek(0)
                m = ss.read(4)
            if m != self.BGZF_MAGIC:
                self.close()
                raise HbamError(E_FORMAT, "Does not seem like a BAM file")

    def guessNextBAMRecordStart(self, beg, end):
        """The virtual offset of the first BAM record in [beg, end), or end."""
        return self._f.guess_record_starts([beg], [end], self._n_ref)[0]

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Gpu:
    """Device-resident pipeline session (bench.py / multi-GPU shards)."""

    def __init__(self, device=0):
        self._h = P()
        rc = _L.hbam_gpu_create(device, C.byref(self._h))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(None).decode())

    def close(self):
        if self._h:
            _L.hbam_gpu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, data):
        """Make a whole BAM resident in HBM (header parsed)."""
        if isinstance(data, np.ndarray):
            ptr, n = data.ctypes.data, data.nbytes
            self._keep = data
        else:
            self._keep = C.create_string_buffer(bytes(data), len(data))
            ptr, n = self._keep, len(data)
        rc = _L.hbam_gpu_load(self._h, ptr, n)
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        self._keep = None

    def set_window(self, window_bytes):
        _L.hbam_gpu_set_window(self._h, window_bytes)

    def run(self, timing=False, decode=True, digest=False):
        st = GpuStats()
        flags = (1 if timing else 0) | (0 if decode else 2) | (4 if digest else 0)
        rc = _L.hbam_gpu_run(self._h, flags, C.byref(st))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return _stats_dict(st)

    def index(self, granularity=4096):
        """.splitting-bai of the resident file: (bytes, ms)."""
        p = P()
        n = u64()
        ms = C.c_float()
        rc = _L.hbam_gpu_index(self._h, granularity, C.byref(p), C.byref(n), C.byref(ms))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        b = C.string_at(p, n.value)
        _L.hbam_free(p)
        return b, ms.value

    def run_streamed(self, ptr, nbytes, piece_bytes=64 << 20):
        """hbam_gpu_run_streamed: copy the file from host memory at `ptr` in
        pieces while inflating the pieces already in HBM, then chain + decode."""
        st = GpuStats()
        rc = _L.hbam_gpu_run_streamed(self._h, ptr, nbytes, piece_bytes, C.byref(st))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return _stats_dict(st)

    def reload(self, ptr, nbytes, pinned=True):
        """Host->HBM copy of the loaded file's bytes from `ptr` (through a
        page-locked staging copy if pinned), timed: milliseconds."""
        ms = C.c_float()
        rc = _L.hbam_gpu_reload(self._h, ptr, nbytes, int(pinned), C.byref(ms))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return ms.value

    def d2d_bandwidth(self, nbytes=1 << 32, iters=5):
        gbps = C.c_float()
        rc = _L.hbam_gpu_d2d_bandwidth(self._h, nbytes, iters, C.byref(gbps))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return gbps.value

    def encode_writables(self, iters=10):
        """SAMRecordWritable.write of the last run's records into device
        memory, timed over `iters` launches: (ms per encode, bytes)."""
        ms = C.c_float()
        nb = u64()
        rc = _L.hbam_gpu_encode_writables(self._h, iters, C.byref(ms), C.byref(nb))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return ms.value, nb.value

    def fetch_encoded(self, pos, length):
        buf = C.create_string_buffer(max(length, 1))
        rc = _L.hbam_gpu_fetch_encoded(self._h, pos, length, buf)
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return buf.raw[:length]

    def bgzf_compress(self, level=5, eof=True, iters=0):
        """BGZF-compress the last run's inflated stream with the loaded file's
        block boundaries (hbam_gpu_bgzf_compress): (ms per compress, bytes)."""
        ms = C.c_float()
        nb = u64()
        rc = _L.hbam_gpu_bgzf_compress(self._h, level, BGZF_EOF if eof else 0, iters, C.byref(ms), C.byref(nb))
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return ms.value, nb.value

    def fetch_compressed(self, pos, length):
        buf = np.empty(max(length, 1), np.uint8)
        rc = _L.hbam_gpu_fetch_compressed(self._h, pos, length, buf.ctypes.data)
        if rc != OK:
            raise HbamError(rc, _L.hbam_gpu_error(self._h).decode())
        return buf[:length]

    def fetch(self, n):
        keys = np.zeros(max(n, 1), np.int64)
        voffs = np.zeros(max(n, 1), np.uint64)
        rc = _L.hbam_gpu_fetch(self._h, keys.ctypes.data, voffs.ctypes.data, n)
        if rc != OK:
            raise HbamError(rc, "fetch failed")
        return keys[:n], voffs[:n]
