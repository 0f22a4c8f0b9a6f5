// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// BAMSplitGuesser on the MI355X read path, with the reference's public API
// (BAMSplitGuesser.java:80-235, 340-401):
//
//   GpuBAMSplitGuesser(SeekableStream, Configuration)                :80-91
//       the stream must hold a BAM file: its header is read from it, and its
//       first four bytes must be the BGZF magic (SAMFormatException)
//   GpuBAMSplitGuesser(SeekableStream, InputStream headerStream, Configuration)
//                                                                    :93-103
//       the header read from another stream (SAMHeaderReader, as the
//       reference): its sequence dictionary bounds the refIDs a guessed
//       record may hold
//   guessNextBAMRecordStart(beg, end)                                :108-235
//       the virtual offset of the first BAM record in [beg, end), or end
//
// BAMSplitGuesser.main (:340-401), a command-line probe, is not mirrored: the
// CLI is outside the read path this class replaces.
//
// The stream is read through hbam_open_reader: a positioned reader over the
// SeekableStream (seek + read, one call at a time), so any Hadoop
// FileSystem's stream works, and only the bytes a guess needs are read
// (MAX_BYTES_READ after beg, as the reference).  The BGZF block search, the
// inflate and the BLOCKS_NEEDED_FOR_GUESS record checks run in gfx950 kernels
// (hbam_guess.hip).  Callers that guess many split points of one file at once
// (BAMInputFormat.getSplits) use HbamNative.guessRecordStarts directly, as
// GpuBAMInputFormat does: one launch per window of nearby points.
//
// The ctx lives until close(); a guesser that is not closed frees it when it
// is finalized (the reference holds no native resources, so its callers
// never close it; Java 8, as the reference's pom, has no Cleaner).
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.SAMFileHeader;
import htsjdk.samtools.SAMFormatException;
import htsjdk.samtools.seekablestream.SeekableStream;
import java.io.Closeable;
import java.io.IOException;
import java.io.InputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.apache.hadoop.conf.Configuration;
import org.seqdoop.hadoop_bam.gpu.HbamNative;
import org.seqdoop.hadoop_bam.util.SAMHeaderReader;

public class GpuBAMSplitGuesser extends BaseSplitGuesser implements Closeable {
  /** As BAMSplitGuesser.MAX_BYTES_READ (:72-73): 3 * 0xffff + 0xfffe. */
  static final int MAX_BYTES_READ = 3 * 0xffff + 0xfffe;

  private long ctx;              // 0 once closed
  private final int headerNRef;  // -1: the data file's own header

  /** One positioned read at a time over the guesser's stream (seek + read). */
  private static final class SeekableReader implements HbamNative.PositionedReader {
    private final SeekableStream ss;
    private final byte[] chunk = new byte[1 << 20];

    SeekableReader(SeekableStream ss) {
      this.ss = ss;
    }

    @Override
    public synchronized int read(long position, ByteBuffer dst) throws IOException {
      ss.seek(position);
      int done = 0;
      final int want = dst.capacity();
      while (done < want) {
        final int r = ss.read(chunk, 0, Math.min(chunk.length, want - done));
        if (r < 0) break;
        dst.put(chunk, 0, r);
        done += r;
      }
      return done == 0 && want > 0 ? -1 : done;
    }
  }

  public GpuBAMSplitGuesser(SeekableStream ss, Configuration conf) throws IOException {
    this(ss, ss, conf);
    // :86-90 the secondary check that the stream holds a BGZF (BAM) file
    final byte[] m = new byte[4];
    ss.seek(0);
    if (ss.read(m, 0, 4) != 4 || ByteBuffer.wrap(m).order(ByteOrder.LITTLE_ENDIAN).getInt() != BGZF_MAGIC) {
      close();
      throw new SAMFormatException("Does not seem like a BAM file");
    }
  }

  public GpuBAMSplitGuesser(SeekableStream ss, InputStream headerStream, Configuration conf) throws IOException {
    in = ss;
    if (headerStream == ss) {
      headerNRef = -1;  // the ctx reads the same header from the data
    } else {
      final SAMFileHeader header = SAMHeaderReader.readSAMHeaderFrom(headerStream, conf);
      headerNRef = header.getSequenceDictionary().size();
    }
    // the guesser's record checks do not depend on the stringency (the
    // reference decodes with its own codec, no SAMRecord.isValid)
    ctx = HbamNative.openReader(ss.length(), new SeekableReader(ss), false, GpuBAMRecordReader.device(conf), false,
                                HbamNative.SILENT, 0, 0);
  }

  /**
   * Finds a virtual BAM record position in the physical position range
   * [beg,end). Returns end if no BAM record was found.
   */
  public long guessNextBAMRecordStart(long beg, long end) throws IOException {
    synchronized (this) {  // close() may race a guess
      if (ctx == 0) throw new IOException("GpuBAMSplitGuesser is closed");
      return HbamNative.guessRecordStartsHdr(ctx, headerNRef, new long[] {beg}, new long[] {end})[0];
    }
  }

  /** Releases the GPU context (HBM windows, page-locked buffers). */
  @Override
  public synchronized void close() {
    if (ctx != 0) HbamNative.close(ctx);
    ctx = 0;
  }

  @Override
  protected void finalize() throws Throwable {
    try {
      close();
    } finally {
      super.finalize();
    }
  }
}
