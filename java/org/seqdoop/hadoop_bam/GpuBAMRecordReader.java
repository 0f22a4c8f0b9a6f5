// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// BAMRecordReader on the MI355X read path (libhbam.so through HbamNative).
// Same contract as BAMRecordReader (BAMRecordReader.java:63-233): key =
// getKey(record) (refIdx << 32 | alignmentStart0, MurmurHash3 branch for
// unmapped reads), value = a BAMRecord in a SAMRecordWritable, records
// of the FileVirtualSplit [vStart, vEnd) in file order, getProgress from the
// stream position htsjdk's iterator would stand at.
//
// What moves to the GPU: BGZF block discovery, inflate, the record chain, the
// htsjdk validation rules of the configured stringency and the 11 fixed
// fields + key + voff of every record (hbam_decode_span, in batches).  What
// stays here: building the record object of each record from the batch's
// columns, exactly the arguments htsjdk's BAMRecordCodec.decode passes to
// SAMRecordFactory.createBAMRecord.  The reference's reader opens its
// SamReader with no record factory (BAMRecordReader.java:186-200), so its
// values are htsjdk's DefaultSAMRecordFactory BAMRecords, and so are these
// (class and reference-name resolution included); the writable codec keeps
// LazyBAMRecordFactory (LazyBAMRecordFactory.java:37-50), as
// SAMRecordWritable's readFields does (SAMRecordWritable.java:47-48).
// With hadoopbam.gpu.encode-writables the values are GpuSAMRecordWritables
// that also carry their SAMRecordWritable.write bytes, encoded per batch on
// the GPU (hbam_encode_writables).
//
// Bounded traversal (intervals / unmapped-only, BAMRecordReader.java:170-178)
// is outside the GPU path: such splits are read by the stock BAMRecordReader
// (GpuBAMInputFormat.createRecordReader).
//
// Not compiled in this repository (no JDK in the build image); it binds the
// native methods of HbamNative exactly as declared there.
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.DefaultSAMRecordFactory;
import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SAMRecord;
import htsjdk.samtools.SAMRecordFactory;
import htsjdk.samtools.ValidationStringency;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;
import org.seqdoop.hadoop_bam.gpu.HbamFiles;
import org.seqdoop.hadoop_bam.gpu.HbamNative;
import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public class GpuBAMRecordReader extends RecordReader<LongWritable, SAMRecordWritable> {
  /** Records per hbam_decode_span batch (hadoopbam.gpu.batch-records). */
  public static final String BATCH_RECORDS_PROPERTY = "hadoopbam.gpu.batch-records";
  public static final String DEVICE_PROPERTY = "hadoopbam.gpu.device";
  public static final String WINDOW_BYTES_PROPERTY = "hadoopbam.gpu.window-bytes";

  private final LongWritable key = new LongWritable();
  // SamReaderFactory.makeDefault()'s factory: BAMRecordReader.createSamReader sets none
  private final SAMRecordFactory factory = DefaultSAMRecordFactory.getInstance();
  // a GpuSAMRecordWritable carrying its record's writable bytes when
  // hadoopbam.gpu.encode-writables is set (GpuSAMRecordWritable.java)
  private SAMRecordWritable record = new SAMRecordWritable();
  private boolean encode;
  private GpuSAMRecordWritable.EncodedBatch encoded;  // the current batch's writable bytes

  private HbamFiles.Handle file;  // the open ctx (and its stream on a non-local file system)
  private long ctx;  // file.ctx, 0 when closed
  private SAMFileHeader header;
  private ValidationStringency stringency;
  private boolean isInitialized = false;
  private boolean reachedEnd;
  private long fileStart, virtualEnd;
  private long batchRecords;

  // the current batch (HbamNative.decodeSpan column order) and the cursor
  private ByteBuffer[] cols;
  private int n, i;  // records in the batch, next record to hand out
  private final long[] cursor = new long[1];
  private boolean started;  // a record has been handed out

  /** Device ordinal: hadoopbam.gpu.device, else LOCAL_RANK (one process per GPU), else 0. */
  static int device(Configuration conf) {
    final String lr = System.getenv("LOCAL_RANK");
    return conf.getInt(DEVICE_PROPERTY, lr == null ? 0 : Integer.parseInt(lr));
  }

  static int stringencyCode(ValidationStringency s) {
    if (s == ValidationStringency.LENIENT) return HbamNative.LENIENT;
    if (s == ValidationStringency.SILENT) return HbamNative.SILENT;
    return HbamNative.STRICT;  // htsjdk's default
  }

  /** The property's stringency, htsjdk's default (STRICT) when unset, as the SamReader applies it. */
  static ValidationStringency stringencyOf(Configuration conf) {
    final ValidationStringency s = SAMHeaderReader.getValidationStringency(conf);
    return s == null ? ValidationStringency.DEFAULT_STRINGENCY : s;
  }

  @Override
  public void initialize(InputSplit spl, TaskAttemptContext tctx) throws IOException {
    // as BAMRecordReader.initialize (:123-184): may be called twice
    if (isInitialized) close();
    isInitialized = true;
    reachedEnd = false;

    final Configuration conf = tctx.getConfiguration();
    final FileVirtualSplit split = (FileVirtualSplit) spl;
    final Path path = split.getPath();

    stringency = stringencyOf(conf);
    header = SAMHeaderReader.readSAMHeaderFrom(path, conf);

    if (conf.getBoolean("hadoopbam.bam.keep-paired-reads-together", false))
      throw new IllegalArgumentException("Property hadoopbam.bam.keep-paired-reads-together is no longer honored.");

    final long virtualStart = split.getStartVirtualOffset();
    fileStart = virtualStart >>> 16;
    virtualEnd = split.getEndVirtualOffset();
    batchRecords = conf.getLong(BATCH_RECORDS_PROPERTY, 1L << 20);
    encode = conf.getBoolean(GpuSAMRecordWritable.ENCODE_PROPERTY, false);
    record = encode ? new GpuSAMRecordWritable() : new SAMRecordWritable();

    // the file through its own file system, as WrapSeekable.openPath (:147):
    // a local path is read with pread, HDFS and the rest through positioned
    // reads of the FSDataInputStream (hbam_open_reader)
    file = HbamFiles.open(path, conf, device(conf), stringencyCode(stringency),
                          conf.getLong(WINDOW_BYTES_PROPERTY, 0L), batchRecords);
    ctx = file.ctx;
    cursor[0] = virtualStart;
    cols = null;
    n = i = 0;
    started = false;
    // htsjdk's iterator reads the first record when it is created
    // (bamFileReader.getIterator, :181-182): so does the first batch here,
    // and a first record that fails validation throws from initialize too
    nextBatch();
  }

  private void nextBatch() throws IOException {
    cols = HbamNative.decodeSpan(ctx, cursor[0], virtualEnd, batchRecords, cursor);
    for (ByteBuffer b : cols) b.order(ByteOrder.LITTLE_ENDIAN);
    n = cols[HbamNative.KEY].capacity() / 8;
    i = 0;
    // hbam_encode_writables encodes the last decodeSpan batch: now, before the next call
    if (encode && n > 0) encoded = GpuSAMRecordWritable.EncodedBatch.of(ctx, n, encoded);  // reuses its buffer
  }

  @Override
  public void close() throws IOException {
    if (file != null) {
      file.close();
      file = null;
      ctx = 0;
    }
    cols = null;
    encoded = null;
  }

  /**
   * As BAMRecordReader.getProgress (:209-219): the stream position htsjdk's
   * iterator stands at (it has read one record ahead), hbam_reader_position.
   */
  @Override
  public float getProgress() throws IOException {
    if (reachedEnd) return 1;
    if (n == 0) return 0;  // an empty split before nextKeyValue has seen its end
    // i - 1: the record nextKeyValue returned last; -1 (UINT64_MAX): none yet
    final long filePos = HbamNative.readerPosition(ctx, started ? i - 1 : -1L);
    final long fileEnd = virtualEnd >>> 16;
    return (float) (filePos - fileStart) / (fileEnd - fileStart + 1);
  }

  @Override
  public LongWritable getCurrentKey() { return key; }

  @Override
  public SAMRecordWritable getCurrentValue() { return record; }

  /**
   * As BAMRecordReader.nextKeyValue (:223-232).  A record failing validation
   * under STRICT/LENIENT ends the batch before it; the next decodeSpan throws
   * the htsjdk exception (SAMFormatException) when the reader reaches it.
   */
  @Override
  public boolean nextKeyValue() throws IOException {
    if (reachedEnd) return false;
    if (i == n) {
      if (n == 0 || cursor[0] >= virtualEnd) {  // the split is done
        reachedEnd = true;
        return false;
      }
      nextBatch();
      if (n == 0) {
        reachedEnd = true;
        return false;
      }
    }
    key.set(cols[HbamNative.KEY].getLong(8 * i));
    final SAMRecord r = recordAt(cols, i, header, factory);
    r.setValidationStringency(stringency);
    if (encoded != null) ((GpuSAMRecordWritable) record).setEncoded(r, encoded, i);
    else record.set(r);
    ++i;
    started = true;
    return true;
  }

  /**
   * The record htsjdk's BAMRecordCodec.decode builds with factory for record
   * j of a batch (decodeSpan or decodeWritables columns): the reader's
   * default-factory BAMRecord, or the writable codec's LazyBAMRecord with
   * header null as SAMRecordWritable's lazyCodec (SAMRecordWritable.java:47-48).
   */
  static SAMRecord recordAt(ByteBuffer[] cols, int j, SAMFileHeader header, SAMRecordFactory factory) {
    final ByteBuffer data = cols[HbamNative.DATA];
    final long off = cols[HbamNative.REST_OFF].getLong(8 * j);
    final int len = cols[HbamNative.REST_LEN].getInt(4 * j);
    final byte[] rest = new byte[len];
    final ByteBuffer d = data.duplicate();
    d.position((int) off);
    d.get(rest, 0, len);
    final SAMRecord r = factory.createBAMRecord(
        header,
        cols[HbamNative.REF_ID].getInt(4 * j),
        cols[HbamNative.POS].getInt(4 * j) + 1,                       // 1-based, as the codec
        (short) (cols[HbamNative.L_READ_NAME].get(j) & 0xff),
        (short) (cols[HbamNative.MAPQ].get(j) & 0xff),
        cols[HbamNative.BIN].getShort(2 * j) & 0xffff,
        cols[HbamNative.N_CIGAR].getShort(2 * j) & 0xffff,
        cols[HbamNative.FLAG].getShort(2 * j) & 0xffff,
        cols[HbamNative.L_SEQ].getInt(4 * j),
        cols[HbamNative.NEXT_REF_ID].getInt(4 * j),
        cols[HbamNative.NEXT_POS].getInt(4 * j) + 1,
        cols[HbamNative.TLEN].getInt(4 * j),
        rest);
    return r;
  }

  /** The BGZF virtual offset of the record last handed out (FileVirtualSplit coordinates). */
  public long getCurrentVirtualOffset() {
    return cols[HbamNative.VOFF].getLong(8 * (i - 1));
  }
}
