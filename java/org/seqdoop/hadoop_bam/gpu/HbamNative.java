// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// JNI facade over libhbam.so (include/hbam.h), the drop-in boundary of the
// MI355X BAM read path.  One handle per opened file (a BAMRecordReader, a
// SplittingBAMIndexer run, a BAMInputFormat planning call).  The Hadoop-BAM
// classes keep their public API and delegate their hot loops here when
// hadoopbam.gpu.enable is true (INTEGRATION.md section 2):
//
//   BAMRecordReader.initialize / nextKeyValue / getProgress
//       (BAMRecordReader.java:123-184, 223-232, 209-219)  -> open, decodeSpan, readerPosition
//       (the delegating classes: ../GpuBAMRecordReader.java, ../GpuBAMInputFormat.java,
//        ../GpuSplittingBAMIndexer.java)
//   SplittingBAMIndexer.index (SplittingBAMIndexer.java:248-290) -> splittingIndex
//   SplittingBAMIndexer.processAlignment + finish (:186-202, 240-243)
//       (write time, BAMRecordWriter.java:131-149)       -> splittingIndexForRecords
//   BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:108-235) -> guessRecordStarts
//   BAMInputFormat.getSplits per file (BAMInputFormat.java:222-318, 469-530) -> getSplits
//   SAMRecordWritable.write / readFields (SAMRecordWritable.java:55-68) -> encodeWritables, decodeWritables
//   BlockCompressedOutputStream under BAMRecordWriter                 -> bgzfCompress
//
// Errors: every native method throws the exception the Java method it
// replaces throws (hbam_jni.c throw_for): HBAM_E_FORMAT -> SAMFormatException,
// HBAM_E_TRUNC -> FileTruncatedException, HBAM_E_ARG -> IllegalArgumentException,
// others -> IOException.
//
// Not compiled in this repository (the build image has no JDK); the same ABI
// is exercised through ctypes by every test (hadoop-bam_amd/hbam/__init__.py).
package org.seqdoop.hadoop_bam.gpu;

import java.io.IOException;
import java.nio.ByteBuffer;

public final class HbamNative {
  static {
    System.loadLibrary("hbam");
    System.loadLibrary("hbam_jni");
  }

  private HbamNative() {}

  /** hadoopbam.samheaderreader.validation-stringency (util/SAMHeaderReader.java:45-46). */
  public static final int STRICT = 0, LENIENT = 1, SILENT = 2;

  /** Column order of {@link #decodeSpan} / {@link #decodeWritables}. */
  public static final int KEY = 0, VOFF = 1, REF_ID = 2, POS = 3, L_READ_NAME = 4, MAPQ = 5, BIN = 6,
      N_CIGAR = 7, FLAG = 8, L_SEQ = 9, NEXT_REF_ID = 10, NEXT_POS = 11, TLEN = 12, REST_OFF = 13,
      REST_LEN = 14, DATA = 15, N_COLUMNS = 16;

  /**
   * hbam_open: maps the file; only the HBM windows a call needs are copied
   * (a split reads about its own byte range).
   *
   * @param device hadoopbam.gpu.device (HIP ordinal; LOCAL_RANK under one process per GPU)
   * @param stringency STRICT / LENIENT / SILENT
   * @param windowBytes hadoopbam.gpu.window-bytes (compressed bytes per HBM window; 0 = 4 GiB)
   * @param batchRecords hadoopbam.gpu.batch-records the reader will pass to decodeSpan (0 = not
   *     known): its page-locked batch buffers are pinned from the open on
   * @return the ctx handle
   */
  public static native long open(String path, int device, boolean checkCrc, int stringency, long windowBytes,
                                 long batchRecords) throws IOException;

  /**
   * Positioned reads of a file, as PositionedReadable.read(position, buf,
   * off, len) of the FSDataInputStream WrapSeekable.openPath wraps
   * (util/WrapSeekable.java:56-87).  dst is a direct buffer over the
   * library's page-locked memory, valid for this call only; return the bytes
   * put into it (from its position 0; fewer only at the end of the file) or
   * -1 at the end of the file.  Called from library threads (attached by the
   * glue); never twice at once for one ctx unless opened with parallelReads.
   */
  public interface PositionedReader {
    int read(long position, ByteBuffer dst) throws IOException;
  }

  /**
   * hbam_open_reader: the file of length size read through reader (HDFS or
   * any Hadoop FileSystem); otherwise as {@link #open}.  parallelReads: the
   * reader may be called from several library threads at once (positioned
   * reads of an FSDataInputStream are thread-safe).  The ctx holds a global
   * reference to reader until {@link #close}.
   */
  public static native long openReader(long size, PositionedReader reader, boolean parallelReads, int device,
                                       boolean checkCrc, int stringency, long windowBytes, long batchRecords)
      throws IOException;

  public static native void close(long ctx);

  /** hbam_header: {n_ref, l_text, first_record_voff, file_size}. */
  public static native long[] header(long ctx) throws IOException;

  /** hbam_header: the SAM header text (SAMFileHeader as text). */
  public static native String headerText(long ctx) throws IOException;

  /** hbam_prefetch: make file bytes [lo, hi) resident in HBM ahead of decodeSpan. */
  public static native void prefetch(long ctx, long lo, long hi) throws IOException;

  /**
   * hbam_decode_span: at most maxRecords (0 = all) records of FileVirtualSplit
   * [vStart, vEnd) (vStart &lt;= voff &lt; vEnd).  Returns N_COLUMNS direct
   * buffers over ctx-owned pinned host memory (valid until the next call on
   * ctx or close), little-endian, in the order of the column constants; the
   * rest of record i is DATA[REST_OFF[i] .. +REST_LEN[i]).  cursor[0]
   * receives next_voff: pass it as vStart of the next call (&gt;= vEnd when the
   * split is done).  Records before a record that fails validation are
   * delivered; the exception is thrown on the following call, when the reader
   * reaches that record.
   */
  public static native ByteBuffer[] decodeSpan(long ctx, long vStart, long vEnd, long maxRecords, long[] cursor)
      throws IOException;

  /**
   * hbam_reader_position: BAMRecordReader.getProgress's in.position() after
   * record i of the last batch; i = -1: before record 0 is handed out.
   */
  public static native long readerPosition(long ctx, long i) throws IOException;

  /** hbam_build_splitting_index: the .splitting-bai bytes (SplittingBAMIndexer.index). */
  public static native byte[] splittingIndex(long ctx, int granularity) throws IOException;

  /**
   * hbam_splitting_index_for_records: the write-time index of a written file:
   * processAlignment for records at voffs (file order), then finish(fileSize).
   */
  public static native byte[] splittingIndexForRecords(int device, long[] voffs, int granularity, long fileSize)
      throws IOException;

  /** hbam_guess_record_starts: BAMSplitGuesser.guessNextBAMRecordStart for many split points. */
  public static native long[] guessRecordStarts(long ctx, long[] begs, long[] ends) throws IOException;

  /**
   * hbam_guess_record_starts_hdr: the same with the header read from another
   * stream than the data (BAMSplitGuesser(SeekableStream, InputStream,
   * Configuration)); headerNRef = its sequence dictionary size (-1: the data
   * file's own header).
   */
  public static native long[] guessRecordStartsHdr(long ctx, int headerNRef, long[] begs, long[] ends)
      throws IOException;

  /**
   * hbam_get_splits_bai: the FileVirtualSplits of one file's FileSplits, from
   * the .splitting-bai (sbi), else -- when hadoopbam.bam.enable-bai-splitter
   * is set and the file has a .bai (bai) -- the BAI split calculator, else
   * probabilistic.  null for a missing file.  Returns {vStart0, vEnd0, vStart1, ...}.
   */
  public static native long[] getSplits(long ctx, long[] starts, long[] lengths, byte[] sbi, byte[] bai)
      throws IOException;

  /**
   * hbam_encode_writables: SAMRecordWritable.write of every record of the last
   * decodeSpan into out (direct buffer); offs[i] = start of record i, offs[n] =
   * total.  Returns the total (out == null only sizes).
   */
  public static native long encodeWritables(long ctx, ByteBuffer out, long[] offs) throws IOException;

  /** hbam_open_codec: a device context with no file (reduce side). */
  public static native long openCodec(int device) throws IOException;

  /** hbam_decode_writables: readFields of n framed values of buf; columns as decodeSpan (VOFF = -1). */
  public static native ByteBuffer[] decodeWritables(long ctx, ByteBuffer buf, long[] offs) throws IOException;

  /**
   * hbam_bgzf_compress: BGZF bytes of payload cut at blockLens (the writer's
   * flush points) at level; eof appends the 28-byte terminator.
   */
  public static native byte[] bgzfCompress(int device, ByteBuffer payload, int[] blockLens, int level, boolean eof)
      throws IOException;

  /** hbam_get_key: BAMRecordReader.getKey(int, int) (BAMRecordReader.java:114-116). */
  public static native long getKey(int refIdx, int alignmentStart);

  /** hbam_get_key0: BAMRecordReader.getKey0(int, int) (BAMRecordReader.java:119-121). */
  public static native long getKey0(int refIdx, int alignmentStart0);

  /** hbam_murmurhash3: util/MurmurHash3.murmurhash3(byte[], int). */
  public static native long murmurhash3(byte[] key, int seed);

  /**
   * hbam_release_cached_memory: the HBM and page-locked blocks closed readers
   * left in the library's process-wide cache go back to the HIP runtime (no
   * reference counterpart; bind to the executor's shutdown).  Bytes released.
   */
  public static native long releaseCachedMemory();
}
