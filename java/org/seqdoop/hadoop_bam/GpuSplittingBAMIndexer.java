// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// SplittingBAMIndexer on the MI355X read path, with the reference's public
// API (SplittingBAMIndexer.java:64-290).  The .splitting-bai bytes are those
// of the reference: big-endian voffs of the first record and of every
// granularity-th record after it, then fileSize << 16.
//
//   index(InputStream, OutputStream, inputSize, granularity)   :248-290
//       the stream read front to back through hbam_open_reader (a
//       forward-only positioned reader), the records chained on the GPU
//       window by window (hbam_build_splitting_index)
//   index(Path, Configuration, OutputStream, granularity)
//       the same for a file of any Hadoop FileSystem (a local path is read
//       with pread, HDFS through FSDataInputStream positioned reads)
//   run(Configuration) :120-135, main(String[]) :72-110
//       as the reference ("input" / "granularity" properties; GRANULARITY
//       files...), through the GPU index
//   new GpuSplittingBAMIndexer(out[, granularity]) + processAlignment(...) +
//   finish(inputSize)   :154-243, the write-time indexer BAMRecordWriter
//       drives (BAMRecordWriter.java:131-149): the first record and every
//       granularity-th one are written as they arrive, in O(1) memory, as the
//       reference does -- a modulo per record has nothing to gain from a GPU
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.SAMFileSource;
import htsjdk.samtools.SAMFileSpan;
import htsjdk.samtools.SAMRecord;
import java.io.BufferedOutputStream;
import java.io.File;
import java.io.FileInputStream;
import java.io.FileOutputStream;
import java.io.IOException;
import java.io.InputStream;
import java.io.OutputStream;
import java.lang.reflect.InvocationTargetException;
import java.lang.reflect.Method;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.LongBuffer;
import java.util.Arrays;
import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.fs.Path;
import org.seqdoop.hadoop_bam.gpu.HbamFiles;
import org.seqdoop.hadoop_bam.gpu.HbamNative;

public final class GpuSplittingBAMIndexer {
  public static final String OUTPUT_FILE_EXTENSION = SplittingBAMIndexer.OUTPUT_FILE_EXTENSION;
  public static final int DEFAULT_GRANULARITY = SplittingBAMIndexer.DEFAULT_GRANULARITY;

  /** As SplittingBAMIndexer.main (:72-110): GRANULARITY files..., each indexed to file.splitting-bai. */
  public static void main(String[] args) {
    if (args.length <= 1) {
      System.out.println(
          "Usage: GpuSplittingBAMIndexer GRANULARITY [BAM files...]\n\n"
          + "Writes, for each GRANULARITY alignments in a BAM file, its virtual file offset\n"
          + "as a big-endian 64-bit integer into [filename].splitting-bai. The file is\n"
          + "terminated by the BAM file's length, in the same format.");
      return;
    }
    int granularity;
    try {
      granularity = Integer.parseInt(args[0]);
    } catch (NumberFormatException e) {
      granularity = 0;
    }
    if (granularity <= 0) {
      System.err.printf("Granularity must be a positive integer, not '%s'!\n", args[0]);
      return;
    }
    for (final String arg : Arrays.asList(args).subList(1, args.length)) {
      final File f = new File(arg);
      System.out.printf("Indexing %s...", f);
      try {
        index(new FileInputStream(f), new BufferedOutputStream(new FileOutputStream(f + OUTPUT_FILE_EXTENSION)),
              f.length(), granularity);
        System.out.println(" done.");
      } catch (IOException e) {
        System.out.println(" FAILED!");
        e.printStackTrace();
      }
    }
  }

  /**
   * As SplittingBAMIndexer.run (:120-135): the "input" path of the default
   * file system, indexed at "granularity" (DEFAULT_GRANULARITY) into
   * input.splitting-bai.
   *
   * @throws IllegalArgumentException if the "input" property is not set
   */
  public static void run(final Configuration conf) throws IOException {
    final String inputString = conf.get("input");
    if (inputString == null)
      throw new IllegalArgumentException("String property \"input\" path not found in given Configuration");
    final FileSystem fs = FileSystem.get(conf);
    final Path input = new Path(inputString);
    index(input, conf, fs.create(input.suffix(OUTPUT_FILE_EXTENSION)), conf.getInt("granularity", DEFAULT_GRANULARITY));
  }

  /**
   * As SplittingBAMIndexer.index (:248-290): rawIn is read front to back and
   * closed, out receives the index and is closed.
   */
  public static void index(final InputStream rawIn, final OutputStream out, final long inputSize,
                           final int granularity) throws IOException {
    try (HbamFiles.Handle h = HbamFiles.open(rawIn, inputSize, device(), HbamNative.STRICT)) {
      out.write(HbamNative.splittingIndex(h.ctx, granularity));
    } finally {
      out.close();
    }
  }

  /** The index of a file of conf's file systems (local: pread; HDFS: positioned reads). */
  public static void index(final Path input, final Configuration conf, final OutputStream out,
                           final int granularity) throws IOException {
    try (HbamFiles.Handle h = HbamFiles.open(input, conf, GpuBAMRecordReader.device(conf), HbamNative.STRICT, 0L)) {
      out.write(HbamNative.splittingIndex(h.ctx, granularity));
    } finally {
      out.close();
    }
  }

  /** hadoopbam.gpu.device is a Configuration property; with none at hand, LOCAL_RANK or 0. */
  static int device() {
    final String lr = System.getenv("LOCAL_RANK");
    return lr == null ? 0 : Integer.parseInt(lr);
  }

  // ---- the write-time indexer (:154-243) ----
  private final OutputStream out;
  private final ByteBuffer byteBuffer = ByteBuffer.allocate(8);
  private final LongBuffer lb;
  private final int granularity;
  private long count;
  private Method getFirstOffset;

  public GpuSplittingBAMIndexer(final OutputStream out) {
    this(out, DEFAULT_GRANULARITY);
  }

  public GpuSplittingBAMIndexer(final OutputStream out, final int granularity) {
    this.out = out;
    this.lb = byteBuffer.order(ByteOrder.BIG_ENDIAN).asLongBuffer();
    this.granularity = granularity;
  }

  /** As processAlignment(SAMRecord) (:186-195): record 0 and every granularity-th record after it. */
  public void processAlignment(final SAMRecord rec) throws IOException {
    if (count == 0 || (count + 1) % granularity == 0) {
      final SAMFileSource fileSource = rec.getFileSource();
      writeVirtualOffset(getPos(fileSource.getFilePointer()));
    }
    count++;
  }

  /** As processAlignment(long) (:197-202). */
  void processAlignment(final long virtualOffset) throws IOException {
    if (count == 0 || (count + 1) % granularity == 0) writeVirtualOffset(virtualOffset);
    count++;
  }

  /** As writeVirtualOffset (:229-232): one big-endian entry. */
  public void writeVirtualOffset(long virtualOffset) throws IOException {
    lb.put(0, virtualOffset);
    out.write(byteBuffer.array());
  }

  /** As finish (:240-243): inputSize << 16, then close. */
  public void finish(long inputSize) throws IOException {
    writeVirtualOffset(inputSize << 16);
    out.close();
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
