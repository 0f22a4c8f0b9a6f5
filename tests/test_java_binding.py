"""CPU: the committed Java drop-in sources agree with the C ABI they bind.

No JDK exists in this image, so the Java classes and the JNI glue are checked
textually: every native method of HbamNative has its JNI function, every
hbam_* call of the glue is declared in include/hbam.h, and every HbamNative
method the delegating classes (GpuBAMRecordReader, GpuBAMInputFormat,
GpuSplittingBAMIndexer, GpuSAMRecordWritable, GpuBAMRecordWriter) call exists
with that arity."""
import os
import re

import hbam

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "org", "seqdoop", "hadoop_bam")
JNI = os.path.join(ROOT, "java", "jni", "hbam_jni.c")


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def _natives():
    src = _strip_comments(open(os.path.join(JAVA, "gpu", "HbamNative.java")).read())
    out = {}
    for m in re.finditer(r"public static native [\w\[\]]+ (\w+)\(([^)]*)\)", src):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def test_every_native_method_has_its_jni_function():
    natives = _natives()
    assert {"open", "openReader", "decodeSpan", "readerPosition", "splittingIndex", "splittingIndexForRecords",
            "getSplits", "getKey", "getKey0", "murmurhash3"} <= set(natives)
    jni = _strip_comments(open(JNI).read())
    fns = {}
    for m in re.finditer(r"JNIEXPORT [\w\s\*]+ FN\((\w+)\)\(([^)]*)\)", jni):
        fns[m.group(1)] = len(m.group(2).split(",")) - 2  # minus JNIEnv*, jclass
    assert set(natives) == set(fns), (set(natives) ^ set(fns))
    for name, n in natives.items():
        assert fns[name] == n, (name, n, fns[name])


def test_jni_calls_only_declared_entry_points():
    declared = set(hbam.exported_symbols_from_header())
    jni = _strip_comments(open(JNI).read())
    called = set(re.findall(r"\b(hbam_\w+)\s*\(", jni))
    assert called and called <= declared, called - declared


def test_delegating_classes_call_existing_natives():
    natives = _natives()
    seen = set()
    for cls in ("GpuBAMRecordReader.java", "GpuBAMInputFormat.java", "GpuSplittingBAMIndexer.java",
                "GpuSAMRecordWritable.java", "GpuBAMRecordWriter.java", os.path.join("gpu", "HbamFiles.java")):
        src = _strip_comments(open(os.path.join(JAVA, cls)).read())
        assert "package org.seqdoop.hadoop_bam" in src
        for m in re.finditer(r"HbamNative\.(\w+)\(", src):
            name = m.group(1)
            assert name in natives, (cls, name)
            # arity: count top-level commas of the call's argument list
            i, depth, args, cur = m.end(), 1, 0, ""
            while depth:
                ch = src[i]
                depth += ch in "(["
                depth -= ch in ")]"
                if depth == 1 and ch == ",":
                    args += 1
                cur += ch
                i += 1
            nargs = 0 if not cur[:-1].strip() else args + 1
            assert nargs == natives[name], (cls, name, nargs, natives[name])
            seen.add(name)
    # the reader path, the indexer and the planner all go through the boundary
    assert {"open", "openReader", "close", "decodeSpan", "readerPosition", "getSplits", "splittingIndex",
            "encodeWritables", "decodeWritables", "bgzfCompress"} <= seen


def test_reader_mirrors_the_reference_reader_surface():
    src = _strip_comments(open(os.path.join(JAVA, "GpuBAMRecordReader.java")).read())
    assert "extends RecordReader<LongWritable, SAMRecordWritable>" in src
    for meth in ("public void initialize(InputSplit", "public boolean nextKeyValue()", "public float getProgress()",
                 "public LongWritable getCurrentKey()", "public SAMRecordWritable getCurrentValue()",
                 "public void close()"):
        assert meth in src, meth
    # the record is built with the codec's argument order (LazyBAMRecordFactory.java:37-50), by
    # the factory the reference's SamReader uses: none is set (BAMRecordReader.java:186-200), so
    # htsjdk's default BAMRecords
    assert "factory.createBAMRecord(" in src
    assert "SAMRecordFactory factory = DefaultSAMRecordFactory.getInstance()" in src


REF_INDEXER = "/root/reference/src/main/java/org/seqdoop/hadoop_bam/SplittingBAMIndexer.java"


def _public_signatures(src):
    """(name, parameter types) of public methods and constructors."""
    out = set()
    for m in re.finditer(r"public\s+(?:static\s+)?(?:final\s+)?(?:[\w<>\[\]]+\s+)?(\w+)\s*\(([^)]*)\)", src):
        types = tuple(re.sub(r"\bfinal\s+", "", a).split()[0] for a in m.group(2).split(",") if a.strip())
        out.add((m.group(1), types))
    return out


def test_gpu_indexer_has_the_reference_indexer_api():
    """GpuSplittingBAMIndexer offers every public entry point of
    SplittingBAMIndexer (SplittingBAMIndexer.java:72-290) with the same
    parameter types (the deprecated granularity-only constructor aside)."""
    gpu = _strip_comments(open(os.path.join(JAVA, "GpuSplittingBAMIndexer.java")).read())
    if os.path.exists(REF_INDEXER):
        ref = _public_signatures(_strip_comments(open(REF_INDEXER).read()))
        ref = {("GpuSplittingBAMIndexer" if n == "SplittingBAMIndexer" else n, t) for n, t in ref
               if (n, t) != ("SplittingBAMIndexer", ("int",)) and n != "PtrSkipPair"}  # (a private helper class)
    else:  # the reference's list, as read from the file above when it was present
        ref = {("main", ("String[]",)), ("run", ("Configuration",)),
               ("index", ("InputStream", "OutputStream", "long", "int")),
               ("GpuSplittingBAMIndexer", ("OutputStream",)), ("GpuSplittingBAMIndexer", ("OutputStream", "int")),
               ("processAlignment", ("SAMRecord",)), ("writeVirtualOffset", ("long",)), ("finish", ("long",))}
    have = _public_signatures(gpu)
    assert ref <= have, ref - have


def test_write_time_indexer_keeps_o1_state():
    """processAlignment writes record 0 and every granularity-th record as it
    arrives (SplittingBAMIndexer.java:186-202), with a long counter: no voff
    buffer that grows with the file."""
    src = _strip_comments(open(os.path.join(JAVA, "GpuSplittingBAMIndexer.java")).read())
    assert "private long count;" in src
    assert src.count("count == 0 || (count + 1) % granularity == 0") == 2
    assert "long[] voffs" not in src and "Arrays.copyOf" not in src


REF = "/root/reference/src/main/java/org/seqdoop/hadoop_bam"


def test_gpu_guesser_has_the_reference_guesser_api():
    """GpuBAMSplitGuesser offers BAMSplitGuesser's public entry points
    (BAMSplitGuesser.java:80-108): both constructors and the guess, on the
    same base class; it reads through a positioned reader over the
    SeekableStream and guesses through hbam_guess_record_starts_hdr.  The
    reference's command-line main (:340-401) is out of scope and absent."""
    src = _strip_comments(open(os.path.join(JAVA, "GpuBAMSplitGuesser.java")).read())
    assert "class GpuBAMSplitGuesser extends BaseSplitGuesser" in src
    ref_file = os.path.join(REF, "BAMSplitGuesser.java")
    if os.path.exists(ref_file):
        ref = _public_signatures(_strip_comments(open(ref_file).read()))
        ref = {("GpuBAMSplitGuesser" if n == "BAMSplitGuesser" else n, t) for n, t in ref if n != "main"}
    else:  # the reference's list, as read from the file above when it was present
        ref = {("GpuBAMSplitGuesser", ("SeekableStream", "Configuration")),
               ("GpuBAMSplitGuesser", ("SeekableStream", "InputStream", "Configuration")),
               ("guessNextBAMRecordStart", ("long", "long"))}
    have = _public_signatures(src)
    assert ref <= have, ref - have
    assert not any(n == "main" for n, _ in have)
    assert "HbamNative.openReader(" in src and "HbamNative.guessRecordStartsHdr(" in src
    assert "SAMHeaderReader.readSAMHeaderFrom(headerStream, conf)" in src


def test_writable_and_writer_mirror_the_reference_surface():
    """GpuSAMRecordWritable is a SAMRecordWritable (write / readFields of
    SAMRecordWritable.java:55-68 overridden); GpuBAMRecordWriter has
    BAMRecordWriter's constructors, close and writeAlignment
    (BAMRecordWriter.java:61-150), and the key-ignoring writer its write
    (KeyIgnoringBAMRecordWriter.java:63-65)."""
    w = _strip_comments(open(os.path.join(JAVA, "GpuSAMRecordWritable.java")).read())
    assert "class GpuSAMRecordWritable extends SAMRecordWritable" in w
    have = _public_signatures(w)
    assert {("write", ("DataOutput",)), ("readFields", ("DataInput",)), ("set", ("SAMRecord",))} <= have
    r = _strip_comments(open(os.path.join(JAVA, "GpuBAMRecordWriter.java")).read())
    assert "extends RecordWriter<K, SAMRecordWritable>" in r
    if os.path.exists(os.path.join(REF, "BAMRecordWriter.java")):
        ref = _public_signatures(_strip_comments(open(os.path.join(REF, "BAMRecordWriter.java")).read()))
        ref = {("GpuBAMRecordWriter" if n == "BAMRecordWriter" else n, t) for n, t in ref}
    else:  # the reference's list, as read from the file above when it was present
        ref = {("GpuBAMRecordWriter", ("Path", "Path", "boolean", "TaskAttemptContext")),
               ("GpuBAMRecordWriter", ("Path", "SAMFileHeader", "boolean", "TaskAttemptContext")),
               ("GpuBAMRecordWriter", ("OutputStream", "SAMFileHeader", "boolean")),
               ("close", ("TaskAttemptContext",))}
    assert ref <= _public_signatures(r), ref - _public_signatures(r)
    assert "protected void writeAlignment(final SAMRecord rec)" in r
    k = _strip_comments(open(os.path.join(JAVA, "GpuKeyIgnoringBAMRecordWriter.java")).read())
    assert "extends GpuBAMRecordWriter<K>" in k and "public void write(K ignored, SAMRecordWritable rec)" in k
    # the stock stream's cut: BlockCompressedOutputStream's buffer size, htsjdk's default level
    assert "BlockCompressedStreamConstants.DEFAULT_UNCOMPRESSED_BLOCK_SIZE" in r and "Defaults.COMPRESSION_LEVEL" in r
