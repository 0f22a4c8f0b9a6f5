// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// BAMRecordWriter (BAMRecordWriter.java:51-168) with its BGZF stream deflated
// on the MI355X (hbam_bgzf_compress).  Same constructors, same bytes: the
// stock writer encodes each record (BAMRecordCodec.encode) into a
// BlockCompressedOutputStream, which deflates a block every time its buffer
// (DEFAULT_UNCOMPRESSED_BLOCK_SIZE: 65498 bytes in the htsjdk that wrote the
// reference's test.bam) fills, and the partial block at flush, at htsjdk's
// default level.
// This writer appends the same record bytes to a direct buffer of many such
// blocks and deflates the full blocks of it in one GPU call; close() flushes
// the partial block and, as the reference, writes no EOF terminator.
//
// The write-time .splitting-bai (hadoopbam.bam.write-splitting-bai,
// :69-74, 145-149): a record's virtual offset (block address << 16 | offset in
// block) is known once its block is compressed, so the writer keeps the
// buffer offsets of the records in the buffer and hands their voffs to
// GpuSplittingBAMIndexer.processAlignment in order when the buffer is
// deflated; finish(file length) as :137-139.
//
// Values from GpuBAMRecordReader under hadoopbam.gpu.encode-writables carry
// their record's BAM bytes already (GpuSAMRecordWritable): they are copied,
// not re-encoded.
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.BAMRecordCodec;
import htsjdk.samtools.Defaults;
import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SAMRecord;
import htsjdk.samtools.SAMSequenceDictionary;
import htsjdk.samtools.SAMSequenceRecord;
import htsjdk.samtools.SAMTextHeaderCodec;
import htsjdk.samtools.util.BinaryCodec;
import htsjdk.samtools.util.BlockCompressedStreamConstants;
import java.io.DataOutputStream;
import java.io.IOException;
import java.io.OutputStream;
import java.io.StringWriter;
import java.io.Writer;
import java.nio.ByteBuffer;
import java.nio.charset.Charset;
import java.util.Arrays;
import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.mapreduce.RecordWriter;
import org.apache.hadoop.mapreduce.TaskAttemptContext;
import org.seqdoop.hadoop_bam.gpu.HbamNative;
import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public abstract class GpuBAMRecordWriter<K> extends RecordWriter<K, SAMRecordWritable> {
  /** Uncompressed bytes deflated per GPU call (rounded down to whole blocks; default 64 MiB). */
  public static final String BUFFER_BYTES_PROPERTY = "hadoopbam.gpu.write-buffer-bytes";

  /** The stock stream's block: BlockCompressedOutputStream deflates its buffer when this many bytes are in it. */
  static final int BLOCK = BlockCompressedStreamConstants.DEFAULT_UNCOMPRESSED_BLOCK_SIZE;

  private OutputStream origOutput;
  private int device;
  private int level;             // BlockCompressedOutputStream's default (Defaults.COMPRESSION_LEVEL)
  private ByteBuffer payload;    // direct; whole blocks
  private long blockAddress;     // compressed bytes written: the stock stream's getFilePointer() >> 16
  private OutputStream payloadOut;
  private DataOutputStream dataOut;
  private BinaryCodec binaryCodec;
  private BAMRecordCodec recordCodec;
  private GpuSplittingBAMIndexer splittingBAMIndexer;
  private long[] pending = new long[1 << 12];  // buffer offsets of the records in the buffer (indexer only)
  private int npending;

  /** A SAMFileHeader is read from the input Path (:61-75). */
  public GpuBAMRecordWriter(Path output, Path input, boolean writeHeader, TaskAttemptContext ctx) throws IOException {
    this(output, SAMHeaderReader.readSAMHeaderFrom(input, ctx.getConfiguration()), writeHeader, ctx);
  }

  /** As :76-90. */
  public GpuBAMRecordWriter(Path output, SAMFileHeader header, boolean writeHeader, TaskAttemptContext ctx)
      throws IOException {
    final Configuration conf = ctx.getConfiguration();
    init(output.getFileSystem(conf).create(output), header, writeHeader, GpuBAMRecordReader.device(conf),
         conf.getLong(BUFFER_BYTES_PROPERTY, 64L << 20));
    if (conf.getBoolean(BAMOutputFormat.WRITE_SPLITTING_BAI, false)) {
      final Path splittingIndex = BAMInputFormat.getIdxPath(output);
      splittingBAMIndexer = new GpuSplittingBAMIndexer(output.getFileSystem(conf).create(splittingIndex));
    }
  }

  /** As the deprecated :97-102 (no Configuration: device LOCAL_RANK or 0, 64 MiB buffer). */
  @Deprecated
  public GpuBAMRecordWriter(OutputStream output, SAMFileHeader header, boolean writeHeader) throws IOException {
    init(output, header, writeHeader, GpuSplittingBAMIndexer.device(), 64L << 20);
  }

  private void init(OutputStream output, SAMFileHeader header, boolean writeHeader, int device, long bufferBytes)
      throws IOException {
    origOutput = output;
    this.device = device;
    level = Defaults.COMPRESSION_LEVEL;
    final long blocks = Math.max(1, Math.min(bufferBytes, Integer.MAX_VALUE) / BLOCK);
    payload = ByteBuffer.allocateDirect((int) (blocks * BLOCK));
    payloadOut = new PayloadStream();
    dataOut = new DataOutputStream(payloadOut);
    binaryCodec = new BinaryCodec(payloadOut);
    recordCodec = new BAMRecordCodec(header);
    recordCodec.setOutputStream(payloadOut);
    if (writeHeader) writeHeader(header);
  }

  /** As close (:131-143): the partial block is deflated, no EOF terminator, the index finished. */
  @Override
  public void close(TaskAttemptContext ctx) throws IOException {
    deflate(payload.position());
    if (splittingBAMIndexer != null) splittingBAMIndexer.finish(blockAddress);
    origOutput.close();
  }

  /** As writeAlignment (:145-150). */
  protected void writeAlignment(final SAMRecord rec) throws IOException {
    noteRecordStart();
    recordCodec.encode(rec);
  }

  /** writeAlignment of a value: a GpuSAMRecordWritable's GPU-encoded bytes are copied as they are. */
  protected void writeAlignment(final SAMRecordWritable value) throws IOException {
    if (!(value instanceof GpuSAMRecordWritable)) {
      writeAlignment(value.get());
      return;
    }
    noteRecordStart();
    value.write(dataOut);  // the batch's bytes, or BAMRecordCodec.encode of a replaced record
    dataOut.flush();
  }

  private void noteRecordStart() {
    if (splittingBAMIndexer == null) return;
    if (npending == pending.length) pending = Arrays.copyOf(pending, 2 * npending);
    pending[npending++] = payload.position();
  }

  /** As writeHeader (:152-167), into the same stream. */
  private void writeHeader(final SAMFileHeader header) {
    binaryCodec.writeBytes("BAM\001".getBytes(Charset.forName("UTF8")));
    final Writer sw = new StringWriter();
    new SAMTextHeaderCodec().encode(sw, header);
    binaryCodec.writeString(sw.toString(), true, false);
    final SAMSequenceDictionary dict = header.getSequenceDictionary();
    binaryCodec.writeInt(dict.size());
    for (final SAMSequenceRecord rec : dict.getSequences()) {
      binaryCodec.writeString(rec.getSequenceName(), true, true);
      binaryCodec.writeInt(rec.getSequenceLength());
    }
  }

  /**
   * The first len buffered bytes, cut every BLOCK bytes as the stock stream
   * cuts them, deflated on the GPU and written out; the voffs of the records
   * that start in them go to the indexer.
   */
  private void deflate(int len) throws IOException {
    if (len == 0) return;
    final int nblocks = (len + BLOCK - 1) / BLOCK;
    final int[] lens = new int[nblocks];
    Arrays.fill(lens, BLOCK);
    lens[nblocks - 1] = len - (nblocks - 1) * BLOCK;
    final ByteBuffer data = payload.duplicate();
    data.position(0).limit(len);
    final byte[] bgzf = HbamNative.bgzfCompress(device, data.slice(), lens, level, false);
    // each block's address: BSIZE (bytes 16-17 of its header) + 1 is its length
    final long[] start = new long[nblocks];
    for (int k = 0, p = 0; k < nblocks; ++k) {
      start[k] = blockAddress + p;
      p += ((bgzf[p + 16] & 0xff) | (bgzf[p + 17] & 0xff) << 8) + 1;
    }
    origOutput.write(bgzf);
    for (int r = 0; r < npending; ++r) {
      final long u = pending[r];
      splittingBAMIndexer.processAlignment(start[(int) (u / BLOCK)] << 16 | (u % BLOCK));
    }
    npending = 0;
    blockAddress += bgzf.length;
    payload.clear();
  }

  /** The buffer as an OutputStream: full means deflate, as the stock stream deflates a full block. */
  private final class PayloadStream extends OutputStream {
    @Override
    public void write(int b) throws IOException {
      payload.put((byte) b);
      if (!payload.hasRemaining()) deflate(payload.position());
    }

    @Override
    public void write(byte[] b, int off, int len) throws IOException {
      while (len > 0) {
        final int k = Math.min(len, payload.remaining());
        payload.put(b, off, k);
        off += k;
        len -= k;
        if (!payload.hasRemaining()) deflate(payload.position());
      }
    }
  }
}
