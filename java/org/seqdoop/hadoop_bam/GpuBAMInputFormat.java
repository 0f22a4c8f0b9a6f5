// Copyright (c) the hadoop-bam_amd authors.  MIT license (as Hadoop-BAM).
//
// BAMInputFormat with split planning and record reading on the MI355X path
// when hadoopbam.gpu.enable is true (INTEGRATION.md section 2).  Everything
// else -- and bounded traversal (intervals, unmapped-only; BAMInputFormat.java:
// 143-184, 532-680), which the GPU path does not cover -- stays the stock
// BAMInputFormat.
//
//   getSplits(splits, cfg)   BAMInputFormat.getSplits (:222-260): per file,
//       addIndexedSplits (.splitting-bai, :264-318), else with
//       hadoopbam.bam.enable-bai-splitter addBAISplits (.bai, :322-465), else
//       addProbabilisticSplits (:469-530) -- one hbam_get_splits_bai call,
//       record starts guessed on the GPU for all of the file's splits at once
//   createRecordReader       GpuBAMRecordReader (BAMRecordReader on the GPU)
//
// Not compiled in this repository (no JDK in the build image).
package org.seqdoop.hadoop_bam;

import htsjdk.samtools.ValidationStringency;
import java.io.ByteArrayOutputStream;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.io.InputStream;
import java.util.ArrayList;
import java.util.Collections;
import java.util.List;
import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.mapreduce.InputSplit;
import org.apache.hadoop.mapreduce.RecordReader;
import org.apache.hadoop.mapreduce.TaskAttemptContext;
import org.apache.hadoop.mapreduce.lib.input.FileSplit;
import org.seqdoop.hadoop_bam.gpu.HbamFiles;
import org.seqdoop.hadoop_bam.gpu.HbamNative;

public class GpuBAMInputFormat extends BAMInputFormat {
  public static final String GPU_ENABLE_PROPERTY = "hadoopbam.gpu.enable";

  static boolean gpuEnabled(Configuration conf) {
    return conf.getBoolean(GPU_ENABLE_PROPERTY, false) && !isBoundedTraversal(conf) && nativeAvailable();
  }

  /** libhbam and its JNI glue load (else the stock classes serve every file). */
  static boolean nativeAvailable() {
    try {
      HbamNative.getKey0(0, 0);
      return true;
    } catch (UnsatisfiedLinkError | NoClassDefFoundError e) {
      return false;
    }
  }

  @Override
  public RecordReader<LongWritable, SAMRecordWritable> createRecordReader(InputSplit split, TaskAttemptContext ctx)
      throws InterruptedException, IOException {
    if (!gpuEnabled(ctx.getConfiguration())) return super.createRecordReader(split, ctx);
    final RecordReader<LongWritable, SAMRecordWritable> rr = new GpuBAMRecordReader();
    rr.initialize(split, ctx);
    return rr;
  }

  @Override
  public List<InputSplit> getSplits(List<InputSplit> splits, Configuration cfg) throws IOException {
    if (!gpuEnabled(cfg)) return super.getSplits(splits, cfg);
    final List<InputSplit> orig = removeIndexFiles(splits);
    // as the reference: sorted by path, each file's splits handled together
    Collections.sort(orig, (a, b) -> ((FileSplit) a).getPath().compareTo(((FileSplit) b).getPath()));
    final List<InputSplit> out = new ArrayList<InputSplit>(orig.size());
    for (int i = 0; i < orig.size();) {
      final Path file = ((FileSplit) orig.get(i)).getPath();
      int j = i;
      while (j < orig.size() && ((FileSplit) orig.get(j)).getPath().equals(file)) ++j;
      addFileSplits(orig.subList(i, j), file, cfg, out);
      i = j;
    }
    return out;
  }

  private static byte[] readAll(FileSystem fs, Path p) throws IOException {
    try (InputStream in = fs.open(p)) {
      final ByteArrayOutputStream b = new ByteArrayOutputStream();
      final byte[] buf = new byte[1 << 16];
      for (int r; (r = in.read(buf)) > 0;) b.write(buf, 0, r);
      return b.toByteArray();
    } catch (FileNotFoundException e) {
      return null;  // addIndexedSplits / addBAISplits would fail to open it: the next planner runs
    }
  }

  private void addFileSplits(List<InputSplit> fileSplits, Path file, Configuration cfg, List<InputSplit> out)
      throws IOException {
    final FileSystem fs = file.getFileSystem(cfg);
    final int n = fileSplits.size();
    final long[] starts = new long[n], lengths = new long[n];
    for (int k = 0; k < n; ++k) {
      final FileSplit f = (FileSplit) fileSplits.get(k);
      starts[k] = f.getStart();
      lengths[k] = f.getLength();
    }
    final byte[] sbi = readAll(fs, getIdxPath(file));
    byte[] bai = null;
    if (cfg.getBoolean(ENABLE_BAI_SPLIT_CALCULATOR, false)) {
      // as addBAISplits (:339-344): <file>.bai, else <name>.bai in place of .bam
      bai = readAll(fs, getBAIPath(file));
      if (bai == null) bai = readAll(fs, new Path(file.toString().replaceFirst("\\.bam$", ".bai")));
    }
    final ValidationStringency vs = GpuBAMRecordReader.stringencyOf(cfg);
    // the guesser reads the file through its own file system, as
    // WrapSeekable.openPath in addProbabilisticSplits (:476)
    final long[] v;
    try (HbamFiles.Handle h = HbamFiles.open(file, cfg, GpuBAMRecordReader.device(cfg),
                                             GpuBAMRecordReader.stringencyCode(vs), 0L)) {
      v = HbamNative.getSplits(h.ctx, starts, lengths, sbi, bai);
    }
    final int m = v.length / 2;
    for (int k = 0; k < m; ++k) {
      // locations: the FileSplit the virtual split was made from (1:1 unless
      // empty probabilistic splits were merged into their predecessor; then
      // the FileSplit holding its start, as addProbabilisticSplits keeps)
      int src = k;
      if (m != n) {
        final long b = v[2 * k] >>> 16;
        src = 0;
        while (src + 1 < n && starts[src + 1] <= b) ++src;
      }
      out.add(new FileVirtualSplit(file, v[2 * k], v[2 * k + 1], ((FileSplit) fileSplits.get(src)).getLocations()));
    }
  }
}
