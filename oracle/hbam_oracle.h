/*
 * hbam_oracle.h -- CPU restatement of Hadoop-BAM's BAM read path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (libhbam.so) never links it.
 *
 * Reference: /root/reference (huangzhibo/Hadoop-BAM 7.9.2-SNAPSHOT, Java) plus
 * htsjdk 2.13.2 (pom.xml:43), which is NOT vendored in the reference.  Every
 * function cites the reference file:line it follows; htsjdk behaviour is
 * marked [htsjdk] and restated from its published semantics.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - inflate: zlib 1.2.x raw inflate (the library java.util.zip.Inflater
 *     wraps), checked against the fixtures' plain-text twins;
 *   - first-record voff of test.bam == 0x196a (TestBAMSplitGuesser.java:21);
 *   - BGZF block boundaries of the VCF fixtures (TestBGZFSplitGuesser.java:36);
 *   - keys / .splitting-bai: cross-checked against an independent Python
 *     restatement (oracle/py_oracle.py); no reference golden exists.
 */
#ifndef HBAM_ORACLE_H
#define HBAM_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/hbam.h */
#define ORC_OK 0
#define ORC_E_FORMAT 1 /* SAMFormatException */
#define ORC_E_TRUNC 2  /* FileTruncatedException / RuntimeEOFException */
#define ORC_E_ARG 3    /* IllegalArgumentException */
#define ORC_E_IO 4     /* IOException / RuntimeIOException */
#define ORC_E_NOMEM 7

/* [htsjdk] ValidationStringency (hadoopbam.samheaderreader.validation-stringency) */
#define ORC_STRICT 0
#define ORC_LENIENT 1
#define ORC_SILENT 2

typedef struct {
  uint64_t coff;   /* compressed offset of the block in the file */
  uint32_t csize;  /* BSIZE + 1 */
  uint32_t isize;  /* ISIZE footer */
  uint32_t crc;    /* CRC32 footer */
  uint32_t pad;
  uint64_t ustart; /* offset of the block's first byte in the inflated stream */
} orc_block;

typedef struct orc_stream orc_stream;

/* Walk + inflate every BGZF block of a whole file (htsjdk
 * BlockCompressedInputStream.readBlock / BlockGunzipper.unzipBlock) and parse
 * the BAM header (htsjdk BAMFileReader.readHeader; SplittingBAMIndexer.java:292-328).
 * parse_header=0 treats the input as plain BGZF (VCF/BCF fixtures). */
int orc_open(const uint8_t *file, uint64_t len, int check_crc, int parse_header,
             orc_stream **out);
void orc_close(orc_stream *s);
const char *orc_error(const orc_stream *s);

uint64_t orc_nblocks(const orc_stream *s);
const orc_block *orc_blocks(const orc_stream *s);
const uint8_t *orc_data(const orc_stream *s);
uint64_t orc_data_len(const orc_stream *s);
int32_t orc_n_ref(const orc_stream *s);
int32_t orc_l_text(const orc_stream *s);
uint64_t orc_header_end(const orc_stream *s);      /* inflated-stream position */
uint64_t orc_first_record_voff(const orc_stream *s);
uint64_t orc_voff_of(const orc_stream *s, uint64_t pos); /* normalized voff */

/* Decoded records of one span, SoA (LazyBAMRecordFactory.java:37-50 field set). */
typedef struct {
  uint64_t n;
  int32_t *ref_id, *pos, *l_seq, *next_ref_id, *next_pos, *tlen;
  uint8_t *l_read_name, *mapq;
  uint16_t *bin, *n_cigar, *flag;
  int64_t *key;
  uint64_t *voff, *offset; /* offset = inflated-stream position of block_size */
  uint32_t *rest_len;
} orc_records;

/* BAMRecordReader.initialize/nextKeyValue over FileVirtualSplit [vstart,vend)
 * (BAMRecordReader.java:123-232 + [htsjdk] BAMFileReader span iterator). */
int orc_decode_span(orc_stream *s, uint64_t vstart, uint64_t vend, orc_records *out);
/* validation stringency of orc_decode_span (default ORC_STRICT, htsjdk's) */
void orc_set_stringency(orc_stream *s, int stringency);
/* [htsjdk] SAMRecord.isValid restated (strict) or the lazy-decode structure
 * checks only (!strict) for the record whose block_size field is at rec;
 * 1 = invalid.  ref_len may be NULL. */
int orc_record_invalid(const uint8_t *rec, int32_t bs, int32_t n_ref, const int32_t *ref_len, int strict);
void orc_records_free(orc_records *r);

/* SAMRecordWritable.write (SAMRecordWritable.java:55-64) of every record in r
 * ([htsjdk] BAMRecordCodec.encode); data = the inflated stream r->offset
 * indexes.  Returns the total size; out may be NULL; offs has r->n+1 slots. */
uint64_t orc_writable_encode(const uint8_t *data, const orc_records *r, uint8_t *out, uint64_t *offs);
/* SAMRecordWritable.readFields (SAMRecordWritable.java:65-68) for n values
 * framed by offs (value i = buf[offs[i], offs[i+1]), the last ends at len). */
int orc_writable_decode(const uint8_t *buf, uint64_t len, const uint64_t *offs, uint64_t n, orc_records *out);

/* SplittingBAMIndexer.index (SplittingBAMIndexer.java:248-368). */
int orc_splitting_index(orc_stream *s, uint64_t file_size, int32_t granularity,
                        uint8_t **out, uint64_t *out_len);
void orc_free(void *p);

/* MurmurHash3.murmurhash3(byte[],int) (util/MurmurHash3.java:32-102). */
int64_t orc_murmurhash3(const uint8_t *key, uint64_t len, int32_t seed);
/* BAMRecordReader.getKey(SAMRecord) (BAMRecordReader.java:81-111) for an
 * undecoded BAM record. */
int64_t orc_get_key(int32_t ref_id, int32_t pos0, uint16_t flag,
                    const uint8_t *var, uint32_t var_len);

/* BaseSplitGuesser.guessNextBGZFPos (BaseSplitGuesser.java:31-108) over a byte
 * array; returns 1 and fills pos/size if found. */
int orc_guess_bgzf_pos(const uint8_t *arr, uint64_t alen, int32_t p, int32_t end,
                       int32_t *pos, int32_t *size);
/* BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:108-235). */
int orc_guess_record_start(orc_stream *s, const uint8_t *file, uint64_t flen,
                           uint64_t beg, uint64_t end, uint64_t *out);
/* the same with the refIDs bounded by another header's dictionary size
 * (BAMSplitGuesser(ss, headerStream, conf), BAMSplitGuesser.java:93-103) */
int orc_guess_record_start_hdr(orc_stream *s, const uint8_t *file, uint64_t flen, int32_t n_ref, uint64_t beg,
                               uint64_t end, uint64_t *out);

/* BGZFSplitGuesser.guessNextBGZFBlockStart (util/BGZFSplitGuesser.java:64-112)
 * restated for the TestBGZFSplitGuesser pins. */
int64_t orc_guess_next_bgzf_block_start(const uint8_t *file, uint64_t flen,
                                        uint64_t beg, uint64_t end);

/* BAMInputFormat split planning for one file (BAMInputFormat.java:264-318,
 * 469-530).  sbi may be NULL (-> probabilistic splits). */
int orc_get_splits(orc_stream *s, const uint8_t *file, uint64_t flen,
                   const uint64_t *starts, const uint64_t *lengths, uint64_t n,
                   const uint8_t *sbi, uint64_t sbi_len, uint64_t *vstarts,
                   uint64_t *vends, uint64_t *nout);

/* [htsjdk] BlockCompressedOutputStream (write + deflateBlock + writeGzipBlock,
 * close() with the EOF terminator when eof != 0): one zlib raw deflater
 * (level, windowBits -15, memLevel 8 -- java.util.zip.Deflater(level, true)),
 * deflateReset per block, deflate(Z_FINISH) into a 65518-byte buffer; a block
 * that does not finish there goes through the NO_COMPRESSION deflater.
 * block_lens[0..nblk) cut data (their sum = len).  Returns the BGZF byte
 * count (out == NULL only sizes; out needs len+64*nblk+28 bytes at most), or UINT64_MAX on a zlib error. */
uint64_t orc_bgzf_compress(const uint8_t *data, uint64_t len, const uint32_t *block_lens,
                           uint64_t nblk, int level, int eof, uint8_t *out);

/* The restated reader / indexer over a whole file on `threads` host threads
 * (orc_scan.c): mode 0 = BAMRecordReader over [first record, EOF) with the
 * given stringency (record count, xor of keys, sum of voffs); mode 1 =
 * SplittingBAMIndexer.index at granularity g into *sbi (orc_free).
 * max_blocks > 0 reads only the first max_blocks BGZF blocks (a sample).
 * Same results as orc_decode_span / orc_splitting_index, streamed block by
 * block: memory is independent of the file size. */
typedef struct {
  uint64_t records, key_xor, voff_sum, blocks, u_bytes;
  int32_t status, rewalks;
  /* order-sensitive digests over the records in file order (bench parity at
   * 60 GB, where xor / sum would cancel over repeated segments):
   * D = sum_i dmix(x_i) * ORC_DIGEST_P^(n-1-i) mod 2^64, x = key (mode 0)
   * or voff (both modes); dmix = MurmurHash3 fmix64.  Composable:
   * D(A ++ B) = D(A) * P^|B| + D(B). */
  uint64_t key_digest, voff_digest;
  /* mode 0: the same digest of each fixed field, in the order refID, pos,
   * l_read_name, mapq, bin, n_cigar, flag, l_seq, next_refID, next_pos, tlen
   * (signed fields sign-extended to 64 bits), and the zlib crc32 of every
   * record's rest ([36, 4 + block_size)) back to back, with its length */
  uint64_t field_digest[11];
  uint32_t rest_crc, pad;
  uint64_t rest_bytes;
} orc_scan_result;
#define ORC_N_FIELDS 11
#define ORC_DIGEST_P 0x100000001b3ull
int orc_scan(const uint8_t *file, uint64_t len, int threads, int mode, int stringency, int32_t g,
             uint64_t max_blocks, uint8_t **sbi, uint64_t *sbi_len, orc_scan_result *res);
/* mode 0 of orc_scan, also writing every record's key and voff in file order
 * into keys / voffs (room for cap records; ORC_E_NOMEM if more) */
int orc_scan_records(const uint8_t *file, uint64_t len, int threads, int stringency, uint64_t cap, int64_t *keys,
                     uint64_t *voffs, orc_scan_result *res);

/* zlib crc32, for tests */
uint32_t orc_crc32(const uint8_t *p, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
