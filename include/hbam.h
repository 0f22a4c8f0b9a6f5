/*
 * hbam.h -- C ABI of the MI355X-native Hadoop-BAM read path (libhbam.so).
 *
 * This is the boundary a JNI shim behind org.seqdoop.hadoop_bam binds (see
 * INTEGRATION.md and java/).  Plain C: pointers, sizes and status codes only.
 * Every entry point names the reference interface it replaces (paths relative
 * to /root/reference/src/main/java/org/seqdoop/hadoop_bam/).
 *
 * Status codes map 1:1 onto the Java exception a caller must raise:
 *   HBAM_E_FORMAT -> htsjdk.samtools.SAMFormatException
 *   HBAM_E_TRUNC  -> htsjdk.samtools.FileTruncatedException / RuntimeEOFException
 *   HBAM_E_ARG    -> java.lang.IllegalArgumentException
 *   HBAM_E_IO     -> java.io.IOException (RuntimeIOException for bad DEFLATE data)
 *   HBAM_E_DEVICE -> java.io.IOException (HIP runtime failure; never a silent CPU path)
 * The message is available from hbam_last_error(ctx).
 *
 * I/O: a ctx reads the file the way BAMRecordReader reads its split through
 * WrapSeekable (WrapSeekable.java:42-87): opening parses the header only, and
 * a decode copies into HBM just the window of compressed bytes it works on
 * (opts.window_bytes at a time, the next record's position carried from one
 * window to the next).  Device memory is bounded by the window, whatever the
 * file size.  hbam_open maps the path read-only and checks the file's
 * length before each read of it; hbam_open_reader reads through a caller's
 * positioned-read callback (a Hadoop FileSystem stream).  A file that turns
 * out shorter than its length at open (truncated while a ctx is open) fails
 * the call that reads there with HBAM_E_TRUNC, and a read error with
 * HBAM_E_IO, as the reference's stream reads throw (only a truncation that
 * races a copy of a mapped path can still raise SIGBUS).
 *
 * Threading: a ctx is single-threaded (RecordReader contract); the library is
 * re-entrant across ctxs.  Each ctx owns one HIP stream on its device.
 * Ownership: memory returned inside hbam_batch / hbam_header_info belongs to
 * the ctx and stays valid until the next call on that ctx or hbam_close.
 * Buffers returned through uint8_t** are released with hbam_free.
 */
#ifndef HBAM_H
#define HBAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBAM_OK 0
#define HBAM_E_FORMAT 1
#define HBAM_E_TRUNC 2
#define HBAM_E_ARG 3
#define HBAM_E_IO 4
#define HBAM_E_DEVICE 5
#define HBAM_E_STATE 6
#define HBAM_E_NOMEM 7

#define HBAM_ABI_VERSION 6

/* htsjdk ValidationStringency, as util/SAMHeaderReader.java:45-46 reads it */
#define HBAM_STRICT 0  /* htsjdk's default: SAMRecord.isValid errors -> SAMFormatException */
#define HBAM_LENIENT 1 /* errors are logged; records still decoded for the check */
#define HBAM_SILENT 2  /* no validation */

typedef struct hbam_ctx hbam_ctx;

/* Reader options: the hadoopbam.* Configuration properties a JNI shim reads. */
typedef struct hbam_opts {
  int32_t device;        /* hadoopbam.gpu.device: HIP device ordinal (default 0) */
  int32_t check_crc;     /* BlockCompressedInputStream.setCheckCrcs (default 0) */
  int32_t stringency;    /* hadoopbam.samheaderreader.validation-stringency (HBAM_STRICT when unset) */
  int32_t parallel_reads; /* hbam_open_reader: nonzero = the read callback may run on several library
                             threads at once (PositionedReadable positioned reads are thread-safe) */
  uint64_t window_bytes; /* hadoopbam.gpu.window-bytes: compressed bytes per HBM window (0 = 4 GiB) */
  uint64_t batch_records; /* hadoopbam.gpu.batch-records: the max_records the caller will pass to
                             hbam_decode_span (0 = not known); its page-locked batch slots are then
                             allocated on a helper thread from the open on */
} hbam_opts;

/* BAM header summary ([htsjdk] BAMFileReader.readHeader). */
typedef struct hbam_header_info {
  int32_t n_ref;                /* binary reference count (SAMSequenceDictionary size) */
  int32_t l_text;               /* SAM header text length */
  uint64_t first_record_voff;   /* getFilePointerSpanningReads().getFirstOffset() */
  uint64_t file_size;           /* compressed bytes */
  const char *text;             /* l_text bytes, owned by ctx */
} hbam_header_info;

/* A batch of decoded records in SoA form: exactly the argument list of
 * LazyBAMRecordFactory.createBAMRecord (LazyBAMRecordFactory.java:37-50)
 * plus the BAMRecordReader key (BAMRecordReader.java:81-121) and the BGZF
 * virtual offset of each record.  pos / next_pos are the 0-based BAM fields
 * (htsjdk alignmentStart = pos + 1).  The rest of record i (read name, cigar,
 * seq, qual, aux = getVariableBinaryRepresentation()) is
 * data[rest_off[i] .. rest_off[i] + rest_len[i]). */
typedef struct hbam_batch {
  uint64_t n;
  const int32_t *ref_id, *pos, *l_seq, *next_ref_id, *next_pos, *tlen;
  const uint8_t *l_read_name, *mapq;
  const uint16_t *bin, *n_cigar, *flag;
  const int64_t *key;
  const uint64_t *voff, *rest_off;
  const uint32_t *rest_len;
  const uint8_t *data;
  uint64_t data_len;
  int32_t status;      /* status of the record that ended the span early (0 = clean end) */
  int32_t reserved;
  uint64_t next_voff;  /* where the split continues: pass it as vstart of the next call; >= vend when done */
} hbam_batch;

/* Open a BAM file (read-only map; nothing but the header is read) / an
 * in-memory BAM / a plain BGZF file (VCF/BCF payloads: no BAM header).
 * Replaces BAMRecordReader.initialize's SamReader construction
 * (BAMRecordReader.java:142-149,186-200) and SAMHeaderReader.readSAMHeaderFrom
 * (util/SAMHeaderReader.java:57-75). */
int hbam_open(const char *path, const hbam_opts *opts, hbam_ctx **out);
int hbam_open_mem(const void *data, uint64_t len, const hbam_opts *opts, hbam_ctx **out);
int hbam_open_bgzf(const void *data, uint64_t len, const hbam_opts *opts, hbam_ctx **out);
/* Positioned read of a file of a known length: copy file bytes
 * [offset, offset + len) into dst and return the bytes copied (fewer only at
 * the end of the file, 0 there) or a negative value on an I/O error.  This is
 * PositionedReadable.read(position, buffer, offset, length) of the
 * FSDataInputStream that WrapSeekable.openPath wraps (util/WrapSeekable.java:
 * 56-87; BAMRecordReader.java:147, BAMInputFormat.java:476).  dst is
 * page-locked host memory the library owns.  The library calls read from its
 * own threads, one call at a time for one ctx (unless opts->parallel_reads): a JNI binding attaches
 * the calling thread to the JVM.  user is passed through.  With
 * opts->parallel_reads set, the library's copy threads call read at once for
 * disjoint ranges (HDFS DFSInputStream positioned reads are thread-safe). */
typedef int64_t (*hbam_read_fn)(void *user, uint64_t offset, void *dst, uint64_t len);
/* hbam_open for a file read through `read` (HDFS or any Hadoop FileSystem):
 * size = FileStatus.getLen().  user must stay valid until hbam_close. */
int hbam_open_reader(uint64_t size, hbam_read_fn read, void *user, const hbam_opts *opts, hbam_ctx **out);
void hbam_close(hbam_ctx *ctx);
const char *hbam_last_error(hbam_ctx *ctx);
void hbam_free(void *p);
int32_t hbam_abi_version(void);
/* Device (HBM) and page-locked host blocks freed by closed contexts stay in
 * a process-wide cache for the next split of the process (an executor or a
 * reused task JVM reads many); this returns them to the HIP runtime.  Call
 * it with no context open (HbamNative.releaseCachedMemory; no reference
 * counterpart).  Returns the bytes released. */
uint64_t hbam_release_cached_memory(void);

int hbam_header(hbam_ctx *ctx, hbam_header_info *out);
/* reference i of the binary dictionary: name (NUL-terminated, ctx-owned) and length */
int hbam_ref(hbam_ctx *ctx, int32_t i, const char **name, int32_t *length);
/* BGZF block count and inflated size of the whole file (reads every block header) */
int hbam_file_stats(hbam_ctx *ctx, uint64_t *n_blocks, uint64_t *uncompressed_size);
/* host -> HBM bytes this ctx has copied so far (its window loads + prefetch) */
int hbam_bytes_read(hbam_ctx *ctx, uint64_t *bytes);
/* Copy file bytes [lo, hi) into HBM now; later windows inside the range decode
 * from HBM without host reads. */
int hbam_prefetch(hbam_ctx *ctx, uint64_t lo, uint64_t hi);

/* Decode records of FileVirtualSplit [vstart, vend) (vStart inclusive, vEnd
 * exclusive: FileVirtualSplit.java:82-86) exactly as BAMRecordReader.initialize
 * + the nextKeyValue loop would (BAMRecordReader.java:151-154,181-182,223-232),
 * with the ctx's validation stringency.  At most max_records records are
 * returned (0 = every record of the split); out->next_voff is where the next
 * call continues, so a split streams in bounded batches:
 *   for (v = vStart; hbam_decode_span(ctx, v, vEnd, max, &b) == HBAM_OK && b.n; v = b.next_voff) ...
 * A call whose vstart is the previous batch's next_voff continues without
 * re-decoding.  Records before a failing record are returned with out->status
 * set and the call returns that status. */
int hbam_decode_span(hbam_ctx *ctx, uint64_t vstart, uint64_t vend, uint64_t max_records, hbam_batch *out);
/* BAMRecordReader.getProgress's in.position() (BAMRecordReader.java:209-219):
 * the compressed stream position after nextKeyValue returned record i of the
 * last batch (htsjdk's iterator has read one record ahead).  i == UINT64_MAX:
 * the position once the iterator exists and before record 0 of the batch is
 * handed out (the iterator has read record 0 only). */
int hbam_reader_position(hbam_ctx *ctx, uint64_t i, uint64_t *pos);

/* SplittingBAMIndexer.index(in, out, inputSize, granularity)
 * (SplittingBAMIndexer.java:248-290): the .splitting-bai bytes, big-endian u64
 * entries, byte-identical to the reference; the file is streamed through HBM
 * window by window.  *buf released with hbam_free. */
int hbam_build_splitting_index(hbam_ctx *ctx, int32_t granularity, uint8_t **buf, uint64_t *len);
/* Write-time index: new SplittingBAMIndexer(out, granularity), processAlignment
 * for records with virtual offsets voffs[0..n) in file order, then
 * finish(file_size) (SplittingBAMIndexer.java:175-243, driven by
 * BAMRecordWriter.java:145-149).  Entries selected on the GPU. */
int hbam_splitting_index_for_records(const hbam_opts *opts, const uint64_t *voffs, uint64_t n, int32_t granularity,
                                     uint64_t file_size, uint8_t **buf, uint64_t *len);

/* BAMSplitGuesser.guessNextBAMRecordStart(beg, end) (BAMSplitGuesser.java:108-235)
 * for n split points at once (one GPU launch per window of nearby points);
 * out[i] == ends[i] when no record start is found, as in the reference. */
int hbam_guess_record_starts(hbam_ctx *ctx, const uint64_t *begs, const uint64_t *ends, uint64_t n,
                             uint64_t *out);
/* The same with the header read from another stream than the data
 * (BAMSplitGuesser(SeekableStream, InputStream headerStream, Configuration),
 * BAMSplitGuesser.java:93-103): header_n_ref = that header's sequence
 * dictionary size, which bounds the refIDs a guessed record may hold
 * (record.setHeaderStrict(header), :185); < 0 = the data file's header. */
int hbam_guess_record_starts_hdr(hbam_ctx *ctx, int32_t header_n_ref, const uint64_t *begs, const uint64_t *ends,
                                 uint64_t n, uint64_t *out);

/* util/BGZFSplitGuesser.guessNextBGZFBlockStart(beg, end)
 * (util/BGZFSplitGuesser.java:64-112) for n split points at once: the first
 * BGZF block start in [beg, beg + min(end-beg, 0xffff)) whose block lies in
 * the guesser's 2*0xffff-1 byte window and inflates with a good CRC;
 * out[i] == ends[i] when none.  The split search of the BGZF text formats
 * (VCFInputFormat / BCFSplitGuesser); works on a ctx from hbam_open_bgzf. */
int hbam_guess_bgzf_block_starts(hbam_ctx *ctx, const uint64_t *begs, const uint64_t *ends, uint64_t n,
                                 uint64_t *out);

/* BAMInputFormat.getSplits for the FileSplits of one file
 * (BAMInputFormat.java:222-318 addIndexedSplits, 469-530 addProbabilisticSplits).
 * sbi = .splitting-bai bytes or NULL.  vstarts/vends need room for n entries. */
int hbam_get_splits(hbam_ctx *ctx, const uint64_t *starts, const uint64_t *lengths, uint64_t n,
                    const uint8_t *sbi, uint64_t sbi_len, uint64_t *vstarts, uint64_t *vends,
                    uint64_t *nout);
/* The same with the BAI split calculator enabled (hadoopbam.bam.enable-bai-splitter,
 * BAMInputFormat.java:241-257, 322-465): with no usable .splitting-bai, splits
 * come from the linear index of the file's .bai (bai bytes; NULL: no .bai ->
 * probabilistic splits), a split no linear entry starts in getting a guessed
 * start.  At most n splits.  Errors as the reference's: a guesser I/O error
 * inside the BAI planner falls back to probabilistic splits (the IOException
 * getSplits catches, :249-253); a malformed .bai -> HBAM_E_FORMAT (htsjdk's
 * unchecked parse error); where addBAISplits dereferences null (no contig
 * with a linear index, a guessed first split) -> HBAM_E_STATE (the JNI glue
 * throws NullPointerException). */
int hbam_get_splits_bai(hbam_ctx *ctx, const uint64_t *starts, const uint64_t *lengths, uint64_t n,
                        const uint8_t *sbi, uint64_t sbi_len, const uint8_t *bai, uint64_t bai_len,
                        uint64_t *vstarts, uint64_t *vends, uint64_t *nout);

/* ---- SAMRecordWritable codec (map-output serialization for the shuffle) ---- */
/* SAMRecordWritable.write (SAMRecordWritable.java:55-64) of every record of
 * the last hbam_decode_span batch on ctx, computed on the GPU: [htsjdk]
 * BAMRecordCodec.encode of each BAMRecord, back to back (block_size, the fixed
 * fields, the undecoded rest; indexBin written as 0 when refID < 0).  *len
 * receives the total size; out == NULL only sizes.  offs (NULL or n+1
 * entries) receives each record's start, offs[n] = *len.  cap < *len ->
 * HBAM_E_ARG.  A batch from several windows (max_records = 0 over a split
 * longer than a window) -> HBAM_E_STATE: encode bounded batches. */
int hbam_encode_writables(hbam_ctx *ctx, uint8_t *out, uint64_t cap, uint64_t *offs, uint64_t *len);
/* SAMRecordWritable.readFields (SAMRecordWritable.java:65-68) for n serialized
 * values at once: value i = buf[offs[i], offs[i+1]) (the last ends at len), as
 * the shuffle frames them.  Decodes into out like hbam_decode_span (voff =
 * UINT64_MAX: no file position; key = BAMRecordReader.getKey of the record).
 * Stops at the first bad value: too short for block_size (readFields would
 * get a null record) or a short rest -> HBAM_E_TRUNC; block_size < 32 ->
 * HBAM_E_FORMAT; framing outside buf -> HBAM_E_ARG. */
int hbam_decode_writables(hbam_ctx *ctx, const void *buf, uint64_t len, const uint64_t *offs, uint64_t n,
                          hbam_batch *out);
/* A ctx with a device and no file, for reducers that only call
 * hbam_decode_writables. */
int hbam_open_codec(const hbam_opts *opts, hbam_ctx **out);

/* ---- BGZF write path ---- */
#define HBAM_BGZF_EOF 1 /* append the 28-byte BGZF EOF terminator (BlockCompressedOutputStream.close) */
/* [htsjdk] BlockCompressedOutputStream.write + deflateBlock + writeGzipBlock
 * (the compressor BAMRecordWriter.java:131-149 writes through) for a whole
 * payload stream, every block DEFLATEd on the GPU in one launch: one
 * java.util.zip.Deflater(level, nowrap) reset per block, output
 * byte-identical to zlib 1.2.11 (levels 0..9; htsjdk's default is 5); a block
 * that does not fit the 65518-byte compressed buffer is written by the
 * NO_COMPRESSION fallback (one stored block).  Blocks: block_lens[0..n_blocks)
 * (each <= 65536, as BlockCompressedOutputStream.flush cuts them; their sum
 * must be len), or when block_lens is NULL, len cut every block_size bytes.
 * *out (BGZF file bytes) is released with hbam_free. */
int hbam_bgzf_compress(const hbam_opts *opts, const void *data, uint64_t len, const uint32_t *block_lens,
                       uint64_t n_blocks, int32_t block_size, int32_t level, int32_t flags, uint8_t **out,
                       uint64_t *out_len);

/* BGZF block table (coff, csize, isize, ustart) and inflated bytes of the
 * whole file: used by tests and by the BGZF text formats. */
int hbam_blocks(hbam_ctx *ctx, uint64_t *coff, uint32_t *csize, uint32_t *isize, uint64_t *ustart,
                uint64_t cap, uint64_t *n);
int hbam_read_inflated(hbam_ctx *ctx, uint64_t pos, uint64_t len, uint8_t *dst);

/* Static key helpers (BAMRecordReader.getKey0 :119-121, getKey(int,int) :114-116,
 * MurmurHash3.murmurhash3(byte[],int) util/MurmurHash3.java:32-102): scalar API
 * for the SAM/CRAM readers that call getKey; the batch path computes keys on
 * the GPU. */
int64_t hbam_get_key0(int32_t ref_idx, int32_t alignment_start0);
int64_t hbam_get_key(int32_t ref_idx, int32_t alignment_start);
int64_t hbam_murmurhash3(const void *key, uint64_t len, int32_t seed);

/* ---- device-resident decode (benchmark / multi-GPU shard driver) ---- */
typedef struct hbam_gpu_stats {
  uint64_t n_blocks;          /* BGZF blocks located (summed over windows) */
  uint64_t compressed_bytes;  /* C of the span: file bytes from its first block to where it ended, each byte once */
  uint64_t inflated_bytes;    /* U of those blocks (windows overlap by a record's blocks: counted once) */
  uint64_t records;           /* N */
  uint64_t first_voff, last_voff;
  uint64_t key_xor, voff_sum; /* order-independent digests of the keys / voffs */
  float ms_locate, ms_inflate, ms_huff, ms_lz77, ms_chain, ms_decode, ms_total;
  int32_t status;
  int32_t link_fallbacks;     /* record-chain spans that took the exact serial link */
  int32_t inflate_launches;   /* phase A + B launch pairs of this run */
  int32_t link_rewalks;       /* parallel-link re-walk rounds of this run */
  int32_t windows;            /* HBM windows the span was decoded in */
  float ms_tables;            /* k_huff_tables (ms_huff: k_inflate_huff, ms_lz77: k_inflate_lz77) */
  int32_t record_fallbacks;   /* windows whose record lists overflowed (indexer mode, records < 36 bytes):
                               * per-block walks counted and emitted the records instead of the fused pass */
  /* order-sensitive digests (flags bit2): sum over the span's records i of
   * fmix64(x_i) * P^(n-1-i) mod 2^64, x = key / voff, P = HBAM_DIGEST_P;
   * the digests of consecutive spans A, B compose as D(A) * P^|B| + D(B) */
  uint64_t key_digest, voff_digest;
} hbam_gpu_stats;
#define HBAM_DIGEST_P 0x100000001b3ull

/* hbam_decode_span with the records left in HBM (no host copies): counts,
 * digests (flags bit2) and per-stage timings (flags bit0) only; flags bit1
 * skips the field decode (chain + voffs only). */
int hbam_decode_span_device(hbam_ctx *ctx, uint64_t vstart, uint64_t vend, int32_t flags, hbam_gpu_stats *st);

/* Cumulative counters of the ctx's decode pipeline since the open, over every
 * call (reader, indexer, device decodes): out[0] spans that took the exact
 * serial link, out[1] parallel-link re-walk rounds, out[2] windows whose
 * record lists overflowed, so that per-block walks counted and emitted the
 * records (hbam_gpu_stats.record_fallbacks), out[3] inflate launch pairs,
 * out[4] spans that stopped early (an error, EOF at an empty block) with
 * records listed in later blocks, which the stop drops.  Diagnostics: tests
 * assert which path a decode took. */
int hbam_pipeline_counters(hbam_ctx *ctx, uint64_t out[5]);

/* The LZ77 tokens inflate phase A wrote for the blocks of the ctx's current
 * window in its last pass (u32 each: phase A's output bytes / 4).  A
 * measurement helper for the bench's traffic figures (no reference
 * counterpart); synchronous. */
int hbam_inflate_token_count(hbam_ctx *ctx, uint64_t *tokens);

/* The sharded SplittingBAMIndexer.index (SplittingBAMIndexer.java:262-287,
 * SURVEY 8e step 3): the records of FileVirtualSplit [vstart, vend) read
 * under the indexer's rules (readAlignment/fullySkip, :340-368), their count
 * in *n_records and, given the global ordinal of the split's first record,
 * the virtual offsets of those whose ordinal + 1 is a multiple of
 * granularity in *entries (*n_entries of them; hbam_free).  The ranks of a
 * multi-GPU read concatenate their entries in split order between the first
 * record's voff and file_size << 16: byte-identical to index() over the
 * whole file. */
int hbam_splitting_entries(hbam_ctx *ctx, uint64_t vstart, uint64_t vend, int32_t granularity, uint64_t ordinal0,
                           uint64_t **entries, uint64_t *n_entries, uint64_t *n_records);

typedef struct hbam_gpu hbam_gpu;

int hbam_gpu_create(int32_t device, hbam_gpu **out);
void hbam_gpu_destroy(hbam_gpu *g);
const char *hbam_gpu_error(hbam_gpu *g);
/* Make a whole BAM file resident in HBM (copied from host memory) and parse
 * its header. */
int hbam_gpu_load(hbam_gpu *g, const void *data, uint64_t len);
/* HBM window of the decode (default 4 GiB of compressed bytes): a file larger
 * than the window is decoded window by window. */
int hbam_gpu_set_window(hbam_gpu *g, uint64_t window_bytes);
/* One pass of the hot path over the resident file, first record to EOF:
 * BGZF discovery, inflate, record scan, field decode + keys + voffs, window by
 * window (flags as hbam_decode_span_device). */
int hbam_gpu_run(hbam_gpu *g, int32_t flags, hbam_gpu_stats *stats);
/* .splitting-bai of the resident file (SplittingBAMIndexer.index), *ms = HIP-event
 * time of the whole call. */
int hbam_gpu_index(hbam_gpu *g, int32_t granularity, uint8_t **buf, uint64_t *len, float *ms);
/* End-to-end pass from host memory: the file (same bytes/length as the loaded
 * one, one window) is copied host->HBM in pieces of piece_bytes on a copy
 * stream while the BGZF blocks of every landed piece are located and inflated
 * on the compute streams; then the record chain + decode (as hbam_gpu_run).
 * st->ms_total = first copy to last decode.  data should come from
 * hbam_host_alloc (page-locked) for the copies to overlap the kernels. */
int hbam_gpu_run_streamed(hbam_gpu *g, const void *data, uint64_t len, uint64_t piece_bytes, hbam_gpu_stats *st);
/* Page-locked host memory (what a JNI caller would wrap as a direct
 * ByteBuffer for the copy engine); NULL on failure. */
void *hbam_host_alloc(uint64_t bytes);
void hbam_host_free(void *p);
/* Copy the loaded file's bytes (same length) from host memory into HBM again,
 * timed (*ms, HIP events): the host->device leg of a PCIe-inclusive rate.
 * pinned != 0 copies from a page-locked staging copy (made untimed). */
int hbam_gpu_reload(hbam_gpu *g, const void *data, uint64_t len, int32_t pinned, float *ms);
/* Measured hipMemcpy device-to-device bandwidth, (read + write) GB/s. */
int hbam_gpu_d2d_bandwidth(hbam_gpu *g, uint64_t bytes, int32_t iters, float *gbps);
/* SAMRecordWritable.write of every record of the last run's last window into
 * a device buffer owned by g, iters timed times (HIP events on the pipeline
 * stream); hbam_gpu_fetch_encoded copies [pos, pos+len) of it to the host. */
int hbam_gpu_encode_writables(hbam_gpu *g, int32_t iters, float *ms_per_iter, uint64_t *bytes);
int hbam_gpu_fetch_encoded(hbam_gpu *g, uint64_t pos, uint64_t len, uint8_t *dst);
/* BGZF-compress the inflated stream of the last run (one window) on the GPU
 * with the loaded file's block boundaries (hbam_bgzf_compress semantics;
 * iters timed repetitions, HIP events); the result stays in HBM,
 * hbam_gpu_fetch_compressed copies [pos, pos+len) of it to the host.
 * Recompressing a file written by zlib at the same level reproduces it byte
 * for byte. */
int hbam_gpu_bgzf_compress(hbam_gpu *g, int32_t level, int32_t flags, int32_t iters, float *ms_per_iter,
                           uint64_t *out_len);
int hbam_gpu_fetch_compressed(hbam_gpu *g, uint64_t pos, uint64_t len, uint8_t *dst);
/* Copy keys / voffs of the last run's last window to the host (either may be NULL). */
int hbam_gpu_fetch(hbam_gpu *g, int64_t *keys, uint64_t *voffs, uint64_t cap);
int32_t hbam_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* HBAM_H */
