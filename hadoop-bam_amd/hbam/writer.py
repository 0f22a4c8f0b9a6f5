"""The BAM write path's host side: BAMRecordWriter (BAMRecordWriter.java:51-168)
over a BGZF stream deflated on the GPU -- the Python mirror of
java/.../GpuBAMRecordWriter.java, same buffering and same voff rule.

The stock writer encodes each record into htsjdk's BlockCompressedOutputStream,
which deflates its buffer every time it fills (HTSJDK_BLOCK_SIZE bytes) and the
partial block at flush; BAMRecordWriter.close flushes and writes no EOF
terminator (:131-143).  BamWriter appends the same bytes to a buffer of many
such blocks and deflates the full buffer in one hbam_bgzf_compress call.  With
a write-time .splitting-bai (:69-74, 145-149) each record's virtual offset --
its block's address << 16 | its offset in the block, the stock stream's
getFilePointer() before the record -- is known once its block is deflated; the
buffered records' offsets are kept until then and fed to the indexer in order
(SplittingBAMIndexer.processAlignment(long) :197-202: record 0 and every
granularity-th record), finish(file length) at close (:240-243)."""
import struct

from . import HTSJDK_BLOCK_SIZE, bgzf_compress


class SplittingIndexWriter:
    """The write-time SplittingBAMIndexer (:154-243) in O(1) state."""

    def __init__(self, out, granularity=4096):
        self.out, self.granularity, self.count = out, granularity, 0

    def process_alignment(self, voff):
        if self.count == 0 or (self.count + 1) % self.granularity == 0:
            self.out.write(struct.pack(">Q", voff))
        self.count += 1

    def finish(self, input_size):
        self.out.write(struct.pack(">Q", input_size << 16))


class BamWriter:
    """out: a binary file object.  header: the BAM header bytes (magic, text,
    references), written into the same stream as writeHeader does (:152-167);
    None writes none (writeHeader false).  buffer_blocks: stock-stream blocks
    deflated per GPU call (hadoopbam.gpu.write-buffer-bytes / block)."""

    def __init__(self, out, header=None, level=5, buffer_blocks=1024, splitting_bai=None, granularity=4096,
                 block=HTSJDK_BLOCK_SIZE, device=0):
        if buffer_blocks < 1 or not 0 < block <= 65536:
            raise ValueError("buffer_blocks >= 1 and 0 < block <= 65536")
        self.out, self.level, self.block, self.device = out, level, block, device
        self.buf = bytearray(buffer_blocks * block)
        self.pos = 0                # bytes in the buffer
        self.block_address = 0      # compressed bytes written so far
        self.pending = []           # buffer offsets of the buffered records (indexer only)
        self.index = SplittingIndexWriter(splitting_bai, granularity) if splitting_bai is not None else None
        if header:
            self._put(header)

    def write_record(self, rec):
        """writeAlignment (:145-150) of one encoded record (block_size included)."""
        if self.index is not None:
            self.pending.append(self.pos)
        self._put(rec)

    def close(self):
        """close (:131-143): the partial block deflated, no EOF; the index finished."""
        self._deflate(self.pos)
        if self.index is not None:
            self.index.finish(self.block_address)

    def _put(self, b):
        b = memoryview(bytes(b))
        while len(b):
            k = min(len(b), len(self.buf) - self.pos)
            self.buf[self.pos:self.pos + k] = b[:k]
            self.pos += k
            b = b[k:]
            if self.pos == len(self.buf):  # full: deflated now, as the stock stream deflates a full block
                self._deflate(self.pos)

    def _deflate(self, n):
        if n == 0:
            return
        lens = [min(self.block, n - p) for p in range(0, n, self.block)]
        z = bgzf_compress(bytes(self.buf[:n]), block_lens=lens, level=self.level, eof=False, device=self.device)
        starts, p = [], 0
        for _ in lens:  # each block's address: BSIZE (header bytes 16-17) + 1 is its length
            starts.append(self.block_address + p)
            p += int.from_bytes(z[p + 16:p + 18], "little") + 1
        self.out.write(z)
        for u in self.pending:
            self.index.process_alignment(starts[u // self.block] << 16 | u % self.block)
        self.pending = []
        self.block_address += len(z)
        self.pos = 0
