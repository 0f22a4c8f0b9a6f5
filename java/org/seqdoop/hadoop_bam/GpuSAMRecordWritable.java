// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// SAMRecordWritable (SAMRecordWritable.java:46-75) on the MI355X path: the
// same value class, whose per-record Writable contract is served from batches
// the GPU encodes or decodes at once.
//
//   write(DataOutput) :55-65
//       Hadoop calls it once per map output value.  GpuBAMRecordReader (with
//       hadoopbam.gpu.encode-writables) encodes every record of a batch on the
//       GPU right after decodeSpan (hbam_encode_writables: BAMRecordCodec.encode
//       of each record, back to back), and hands out values that carry their
//       record's slice of that buffer.  write copies the slice: the bytes are
//       those the reference's codec writes for the record as read.  A value
//       whose record was replaced with set(...), or changed in place since it
//       was read, encodes through htsjdk, as the reference does: write
//       compares the record's fixed fields with the encoded ones, and htsjdk's
//       BAMRecord drops its variable-length bytes (getVariableBinaryRepresentation
//       returns null) once a setter touches the read name, cigar, bases,
//       qualities or tags.  The batch buffer is one direct buffer per reader,
//       grown when a batch needs more and reused across batches.
//   readFields(DataInput) :66-68
//       one value at a time from a stream: the reference's codec (there is no
//       batch to hand to a device).
//   readAll(codecCtx, framed, offs)
//       readFields of a run of framed values at once (a reduce input segment
//       read into a direct buffer): hbam_decode_writables, then the
//       LazyBAMRecord of each value, as readFields builds it.
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.SAMRecord;
import java.io.DataInput;
import java.io.DataOutput;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.seqdoop.hadoop_bam.gpu.HbamNative;

public class GpuSAMRecordWritable extends SAMRecordWritable {
  /** Encode each reader batch's writable bytes on the GPU (GpuBAMRecordReader values). */
  public static final String ENCODE_PROPERTY = "hadoopbam.gpu.encode-writables";

  /** SAMRecordWritable.write of every record of one reader batch (hbam_encode_writables). */
  public static final class EncodedBatch {
    private final ByteBuffer bytes;  // direct, the records' encodings back to back
    private final long[] offs;       // n + 1 starts; offs[n] = total
    private byte[] scratch = new byte[0];

    private EncodedBatch(ByteBuffer bytes, long[] offs) {
      this.bytes = bytes;
      this.offs = offs;
    }

    /**
     * The last decodeSpan batch of ctx (n records), encoded into prev's
     * direct buffer when it is large enough (the reader's previous batch:
     * its values are dead once the next batch is decoded), else into a new
     * one with room to spare.  Direct buffers are freed only by GC, so one per
     * reader keeps a long split from churning direct memory.
     */
    static EncodedBatch of(long ctx, int n, EncodedBatch prev) throws IOException {
      final long total = HbamNative.encodeWritables(ctx, null, null);  // sizes only
      if (total > Integer.MAX_VALUE)  // the largest direct ByteBuffer: lower hadoopbam.gpu.batch-records
        throw new IOException("encoded batch of " + total + " bytes exceeds a ByteBuffer");
      ByteBuffer b = prev != null ? prev.bytes : null;
      if (b == null || b.capacity() < total)
        b = ByteBuffer.allocateDirect((int) Math.min(Integer.MAX_VALUE, Math.max(total, total + total / 4)));
      b.clear();
      final long[] offs = prev != null && prev.offs.length >= n + 1 ? prev.offs : new long[n + 1];
      HbamNative.encodeWritables(ctx, b, offs);
      final EncodedBatch e = new EncodedBatch(b, offs);
      e.scratch = prev != null ? prev.scratch : e.scratch;
      return e;
    }

    /**
     * Whether r still encodes to record i's bytes: its fixed fields equal
     * the encoded ones (BAMRecordCodec.encode's order after block_size:
     * refID, pos, bin_mq_nl, flag_nc, l_seq, next_refID, next_pos, tlen) and
     * htsjdk still holds its variable-length bytes as read.
     */
    boolean encodes(int i, SAMRecord r) {
      if (r.getVariableBinaryRepresentation() == null) return false;  // a setter made them stale
      final ByteBuffer b = bytes.duplicate().order(ByteOrder.LITTLE_ENDIAN);
      final int o = (int) offs[i] + 4;
      final int ref = b.getInt(o), pos = b.getInt(o + 4), binMqNl = b.getInt(o + 8), flagNc = b.getInt(o + 12);
      final Integer bin = r.getIndexingBin();
      return r.getReferenceIndex() == ref && r.getAlignmentStart() - 1 == pos
          && r.getMappingQuality() == ((binMqNl >>> 8) & 0xff) && r.getFlags() == (flagNc >>> 16)
          && r.getMateReferenceIndex() == b.getInt(o + 20) && r.getMateAlignmentStart() - 1 == b.getInt(o + 24)
          && r.getInferredInsertSize() == b.getInt(o + 28)
          && (ref < 0 || bin == null || bin == (binMqNl >>> 16));
    }

    /** Record i's bytes to out: what SAMRecordWritable.write writes for it. */
    void write(int i, DataOutput out) throws IOException {
      final int off = (int) offs[i], len = (int) (offs[i + 1] - offs[i]);
      if (scratch.length < len) scratch = new byte[Math.max(len, 2 * scratch.length)];
      final ByteBuffer d = bytes.duplicate();
      d.position(off);
      d.get(scratch, 0, len);
      out.write(scratch, 0, len);
    }
  }

  private EncodedBatch batch;  // null: encode through htsjdk
  private int index;
  private SAMRecord encodedRecord;  // the record batch[index] encodes

  /** Record i of a reader batch, with its encoding (GpuBAMRecordReader.nextKeyValue). */
  void setEncoded(SAMRecord r, EncodedBatch b, int i) {
    super.set(r);
    batch = b;
    index = i;
    encodedRecord = r;
  }

  @Override
  public void set(SAMRecord r) {
    super.set(r);
    batch = null;
  }

  /** As SAMRecordWritable.write (:55-65); the batch's bytes when they encode this record as it is now. */
  @Override
  public void write(DataOutput out) throws IOException {
    if (batch != null && get() == encodedRecord && batch.encodes(index, encodedRecord)) batch.write(index, out);
    else super.write(out);
  }

  /** As SAMRecordWritable.readFields (:66-68). */
  @Override
  public void readFields(DataInput in) throws IOException {
    batch = null;
    super.readFields(in);
  }

  /**
   * readFields of n framed values at once: value i = framed[offs[i],
   * offs[i+1]) (the last ends at the buffer's capacity), decoded on the device
   * of codecCtx (HbamNative.openCodec).  The exceptions are readFields's: a
   * value too short for its record -> FileTruncatedException (readFields
   * would leave a null record), block_size &lt; 32 -> SAMFormatException.
   */
  public static SAMRecord[] readAll(long codecCtx, ByteBuffer framed, long[] offs) throws IOException {
    final ByteBuffer[] cols = HbamNative.decodeWritables(codecCtx, framed, offs);
    for (ByteBuffer b : cols) b.order(ByteOrder.LITTLE_ENDIAN);
    final int n = cols[HbamNative.KEY].capacity() / 8;
    final LazyBAMRecordFactory factory = new LazyBAMRecordFactory();
    final SAMRecord[] out = new SAMRecord[n];
    for (int j = 0; j < n; ++j) out[j] = GpuBAMRecordReader.recordAt(cols, j, null, factory);
    return out;
  }
}
