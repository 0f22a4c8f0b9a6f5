// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// SplittingBAMIndexer on the MI355X read path.  The .splitting-bai bytes are
// those of SplittingBAMIndexer (SplittingBAMIndexer.java:64-290): big-endian
// voffs of the first record and of every granularity-th record after it, then
// fileSize << 16.
//
//   index(path, out, inputSize, granularity)   SplittingBAMIndexer.index (:248-290):
//       the whole file decoded on the GPU (hbam_build_splitting_index)
//   new GpuSplittingBAMIndexer(out, g) + processAlignment(...) + finish(size)
//       the write-time indexer (:175-243) driven by BAMRecordWriter
//       (BAMRecordWriter.java:131-149): voffs are buffered and the entries
//       selected on the GPU at finish (hbam_splitting_index_for_records)
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.SAMFileSource;
import htsjdk.samtools.SAMFileSpan;
import htsjdk.samtools.SAMRecord;
import java.io.IOException;
import java.io.OutputStream;
import java.lang.reflect.InvocationTargetException;
import java.lang.reflect.Method;
import java.util.Arrays;
import org.seqdoop.hadoop_bam.gpu.HbamNative;

public final class GpuSplittingBAMIndexer {
  private final OutputStream out;
  private final int granularity;
  private final int device;
  private long[] voffs = new long[1 << 16];
  private int count;
  private Method getFirstOffset;

  public GpuSplittingBAMIndexer(final OutputStream out, final int granularity, final int device) {
    this.out = out;
    this.granularity = granularity;
    this.device = device;
  }

  public GpuSplittingBAMIndexer(final OutputStream out) {
    this(out, SplittingBAMIndexer.DEFAULT_GRANULARITY, 0);
  }

  /** SplittingBAMIndexer.processAlignment(SAMRecord) (:186-195): the record's first file pointer. */
  public void processAlignment(final SAMRecord rec) throws IOException {
    final SAMFileSource fileSource = rec.getFileSource();
    processAlignment(getPos(fileSource.getFilePointer()));
  }

  /** SplittingBAMIndexer.processAlignment(long) (:197-202): every record's voff, in file order. */
  public void processAlignment(final long virtualOffset) {
    if (count == voffs.length) voffs = Arrays.copyOf(voffs, count * 2);
    voffs[count++] = virtualOffset;
  }

  /** SplittingBAMIndexer.finish (:240-243): the entries and fileSize << 16, then close. */
  public void finish(long inputSize) throws IOException {
    final byte[] idx = HbamNative.splittingIndexForRecords(device, Arrays.copyOf(voffs, count), granularity,
                                                           inputSize);
    out.write(idx);
    out.close();
  }

  /** SplittingBAMIndexer.index (:248-290) for a BAM file on a local file system. */
  public static void index(final String bamPath, final OutputStream out, final int granularity, final int device,
                           final int stringency) throws IOException {
    final long ctx = HbamNative.open(bamPath, device, false, stringency, 0L);
    try {
      out.write(HbamNative.splittingIndex(ctx, granularity));
    } finally {
      HbamNative.close(ctx);
      out.close();
    }
  }

  // as SplittingBAMIndexer.getPos (:204-223): BAMFileSpan is package private in htsjdk
  private long getPos(SAMFileSpan filePointer) {
    if (getFirstOffset == null) {
      try {
        getFirstOffset = filePointer.getClass().getDeclaredMethod("getFirstOffset");
        getFirstOffset.setAccessible(true);
      } catch (NoSuchMethodException e) {
        throw new IllegalStateException(e);
      }
    }
    try {
      return (Long) getFirstOffset.invoke(filePointer);
    } catch (IllegalAccessException | InvocationTargetException e) {
      throw new IllegalStateException(e);
    }
  }
}
