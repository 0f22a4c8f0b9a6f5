/*
 * hbam_oracle.c -- CPU restatement of Hadoop-BAM's BAM read path.
 *
 * TEST INFRASTRUCTURE ONLY (see hbam_oracle.h).  Nothing in the product links
 * or calls this file; tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it via ctypes as the checker / CPU baseline.
 *
 * All citations are relative to /root/reference/src/main/java/org/seqdoop/hadoop_bam/
 * unless prefixed.  [htsjdk] marks htsjdk 2.13.2 semantics (third-party,
 * pom.xml:43, not vendored) restated from its published behaviour.
 */
#include "hbam_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

struct orc_stream {
  orc_block *blk;
  uint64_t nblk;
  uint8_t *data;      /* concatenated inflated blocks */
  uint64_t data_len;
  uint64_t file_len;
  int32_t n_ref;
  int32_t l_text;
  uint64_t header_end; /* inflated-stream position after the binary refs */
  int has_header;
  int32_t *ref_len;    /* binary dictionary lengths (STRICT alignment-start checks) */
  int stringency;      /* ORC_STRICT (htsjdk default) / ORC_LENIENT / ORC_SILENT */
  char err[256];
};

static int set_err(orc_stream *s, int code, const char *fmt, ...) {
  if (s) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(s->err, sizeof s->err, fmt, ap);
    va_end(ap);
  }
  return code;
}

static inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline int32_t rdi32(const uint8_t *p) { return (int32_t)rd32(p); }
static inline uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

/* ------------------------------------------------------------------------ */
/* BGZF block framing + inflate.                                             */
/* [htsjdk] BlockCompressedInputStream.readBlock: 18-byte header, BSIZE at    */
/* offset 16, blockLength = BSIZE+1 must be in [18, 65536]; truncated block ->*/
/* FileTruncatedException.  [htsjdk] BlockGunzipper.unzipBlock: ID1 ID2 CM FLG*/
/* = 1f 8b 08 04, XLEN == 6, raw inflate of blockLength-26 bytes into exactly */
/* ISIZE bytes ("Did not inflate expected amount" otherwise), optional CRC.   */
/* Cut-off heuristic twin: BaseSplitGuesser.java:31-108.                      */
/* ------------------------------------------------------------------------ */

/* Parse the block at p; returns status; fills b (without ustart). */
static int parse_block(orc_stream *s, const uint8_t *f, uint64_t n, uint64_t p, orc_block *b) {
  if (n - p < 18) return set_err(s, ORC_E_IO, "Incorrect header size at %llu", (unsigned long long)p);
  uint32_t total = (uint32_t)rd16(f + p + 16) + 1;
  if (total < 18 || total > 65536)
    return set_err(s, ORC_E_IO, "Unexpected compressed block length %u", total);
  if (p + total > n) return set_err(s, ORC_E_TRUNC, "Premature end of file at block %llu", (unsigned long long)p);
  const uint8_t *h = f + p;
  if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4)
    return set_err(s, ORC_E_FORMAT, "Invalid GZIP header");
  if (rd16(h + 10) != 6) return set_err(s, ORC_E_FORMAT, "Invalid GZIP header");
  if (total < 26) return set_err(s, ORC_E_FORMAT, "block too short for footer");
  b->coff = p;
  b->csize = total;
  b->crc = rd32(h + total - 8);
  b->isize = rd32(h + total - 4);
  b->pad = 0;
  return ORC_OK;
}

/* Raw-DEFLATE inflate into exactly isize bytes ([htsjdk] BlockGunzipper). */
static int inflate_block(orc_stream *s, const uint8_t *f, const orc_block *b, uint8_t *dst, int check_crc) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (inflateInit2(&z, -15) != Z_OK) return set_err(s, ORC_E_NOMEM, "inflateInit2");
  z.next_in = (Bytef *)(f + b->coff + 18);
  z.avail_in = b->csize - 26;
  z.next_out = dst;
  z.avail_out = b->isize;
  int rc = Z_OK;
  while (z.avail_out > 0) {
    rc = inflate(&z, Z_NO_FLUSH);
    if (rc == Z_STREAM_END) break;
    if (rc != Z_OK) break;
    if (z.avail_in == 0) break;
  }
  uint64_t got = b->isize - z.avail_out;
  inflateEnd(&z);
  if (rc != Z_OK && rc != Z_STREAM_END && rc != Z_BUF_ERROR)
    return set_err(s, ORC_E_IO, "DataFormatException in block %llu", (unsigned long long)b->coff);
  if (got != b->isize) return set_err(s, ORC_E_FORMAT, "Did not inflate expected amount");
  if (check_crc) {
    uint32_t c = (uint32_t)crc32(0L, dst, b->isize);
    if (c != b->crc) return set_err(s, ORC_E_FORMAT, "CRC mismatch");
  }
  return ORC_OK;
}

uint32_t orc_crc32(const uint8_t *p, uint64_t n) { return (uint32_t)crc32(0L, p, (uInt)n); }

/* [htsjdk] BlockCompressedOutputStream.deflateBlock / writeGzipBlock (not
 * vendored in the reference; restated from htsjdk 2.13.2's published
 * behaviour): the BGZF writer under BAMRecordWriter.java:131-149. */
uint64_t orc_bgzf_compress(const uint8_t *data, uint64_t len, const uint32_t *block_lens,
                           uint64_t nblk, int level, int eof, uint8_t *out) {
  enum { kCap = 65536 - 18 };
  static const uint8_t eofb[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                   2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  z_stream z, z0;
  memset(&z, 0, sizeof z);
  memset(&z0, 0, sizeof z0);
  if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return UINT64_MAX;
  if (deflateInit2(&z0, 0, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return UINT64_MAX;
  uint8_t *cbuf = (uint8_t *)malloc(kCap);
  uint64_t o = 0, pos = 0;
  (void)len;
  for (uint64_t b = 0; b < nblk; ++b) {
    const uint32_t n = block_lens[b];
    deflateReset(&z);
    z.next_in = (Bytef *)(data + pos);
    z.avail_in = n;
    z.next_out = cbuf;
    z.avail_out = kCap;
    int rc = deflate(&z, Z_FINISH);
    uint32_t cn = kCap - z.avail_out;
    if (rc != Z_STREAM_END) { /* deflater.finished() false -> NO_COMPRESSION deflater */
      deflateReset(&z0);
      z0.next_in = (Bytef *)(data + pos);
      z0.avail_in = n;
      z0.next_out = cbuf;
      z0.avail_out = kCap;
      if (deflate(&z0, Z_FINISH) != Z_STREAM_END) {
        o = UINT64_MAX;
        break;
      }
      cn = kCap - z0.avail_out;
    }
    const uint32_t total = cn + 26;
    if (out) {
      static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
      uint8_t *q = out + o;
      memcpy(q, hdr, 16);
      q[16] = (uint8_t)(total - 1);
      q[17] = (uint8_t)((total - 1) >> 8);
      memcpy(q + 18, cbuf, cn);
      const uint32_t c = (uint32_t)crc32(0L, data + pos, n);
      for (int k = 0; k < 4; ++k) q[18 + cn + k] = (uint8_t)(c >> (8 * k));
      for (int k = 0; k < 4; ++k) q[22 + cn + k] = (uint8_t)(n >> (8 * k));
    }
    o += total;
    pos += n;
  }
  if (o != UINT64_MAX && eof) {
    if (out) memcpy(out + o, eofb, 28);
    o += 28;
  }
  free(cbuf);
  deflateEnd(&z);
  deflateEnd(&z0);
  return o;
}

/* logical stream helpers ------------------------------------------------- */

/* first block index with ustart >= pos */
static uint64_t lower_ustart(const orc_stream *s, uint64_t pos) {
  uint64_t lo = 0, hi = s->nblk;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (s->blk[mid].ustart >= pos) hi = mid; else lo = mid + 1;
  }
  return lo;
}

/* [htsjdk] BlockCompressedInputStream.getFilePointer: (blockAddress<<16)|offset,
 * or (blockAddress+blockLength)<<16 = the address of the NEXT block (empty or
 * not) once the current block is exhausted.  Used for record voffs
 * (BAMFileReader span iterator) and SplittingBAMIndexer.java:263,343. */
uint64_t orc_voff_of(const orc_stream *s, uint64_t pos) {
  uint64_t lo = lower_ustart(s, pos);
  if (lo < s->nblk && s->blk[lo].ustart == pos) return s->blk[lo].coff << 16;
  if (lo == 0) return 0;
  const orc_block *b = &s->blk[lo - 1];
  if (pos - b->ustart < b->isize) return (b->coff << 16) | (pos - b->ustart);
  return (b->coff + b->csize) << 16;
}

/* [htsjdk] read(byte[],..) on an exhausted block calls readBlock(); an empty
 * block makes available()==0 and the call returns -1 (EOF).  Within one read
 * call an empty block only ends the call (partial read) and the next call
 * skips it, so empty blocks are transparent EXCEPT at a position where a new
 * read call starts on an exhausted block: "dead" positions. */
static int dead_at(const orc_stream *s, uint64_t q) {
  uint64_t lo = lower_ustart(s, q);
  return lo > 0 && lo < s->nblk && s->blk[lo].ustart == q && s->blk[lo].isize == 0;
}

/* BAMRecordCodec.decode reads block_size and the fixed fields with separate
 * BinaryCodec calls (readInt/readUByte/readUShort) and the rest with one
 * readBytes: each call start is a potential EOF point. */
static const uint8_t kFieldStarts[] = {4, 8, 12, 13, 14, 16, 18, 20, 24, 28, 32};
static int dead_in_record(const orc_stream *s, uint64_t p, int32_t bs) {
  for (unsigned i = 0; i < sizeof kFieldStarts; i++)
    if (dead_at(s, p + kFieldStarts[i])) return 1;
  return bs > 32 && dead_at(s, p + 36);
}

/* voff -> inflated position; -1 if the pointer is invalid ([htsjdk] seek:
 * "Invalid file pointer" when offset > block length). */
static int64_t pos_of_voff(const orc_stream *s, uint64_t voff) {
  uint64_t coff = voff >> 16, uoff = voff & 0xffff;
  uint64_t lo = 0, hi = s->nblk;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (s->blk[mid].coff >= coff) hi = mid; else lo = mid + 1;
  }
  if (lo >= s->nblk) {
    if (coff == s->file_len && uoff == 0) return (int64_t)s->data_len;
    return -1;
  }
  if (s->blk[lo].coff != coff) return -1;
  if (uoff > s->blk[lo].isize) return -1;
  return (int64_t)(s->blk[lo].ustart + uoff);
}

/* ------------------------------------------------------------------------ */
/* BAM header ([htsjdk] BAMFileReader.readHeader; SplittingBAMIndexer.java:292-328) */
/* ------------------------------------------------------------------------ */
static int parse_header(orc_stream *s) {
  const uint8_t *d = s->data;
  uint64_t end = s->data_len, p = 0;
  if (end < 4) return set_err(s, ORC_E_IO, "Invalid BAM header: too short, no magic");
  if (!(d[0] == 'B' && d[1] == 'A' && d[2] == 'M' && d[3] == 1))
    return set_err(s, ORC_E_IO, "Invalid BAM file header");
  p = 4;
  if (end - p < 4) return set_err(s, ORC_E_TRUNC, "no SAM header length");
  int32_t l_text = rdi32(d + p);
  p += 4;
  if (l_text < 0) return set_err(s, ORC_E_IO, "Invalid BAM header: negative SAM header length %d", l_text);
  if (end - p < (uint64_t)l_text) return set_err(s, ORC_E_TRUNC, "header text truncated");
  p += (uint64_t)l_text;
  if (end - p < 4) return set_err(s, ORC_E_TRUNC, "no reference sequence count");
  int32_t n_ref = rdi32(d + p);
  p += 4;
  free(s->ref_len);
  s->ref_len = (int32_t *)calloc(n_ref > 0 ? (size_t)n_ref : 1, sizeof(int32_t));
  if (!s->ref_len) return set_err(s, ORC_E_NOMEM, "oom");
  for (int32_t i = 0; i < n_ref; i++) {
    if (end - p < 4) return set_err(s, ORC_E_TRUNC, "EOF before reference %d", i + 1);
    int32_t l_name = rdi32(d + p);
    p += 4;
    if (l_name < 0 || end - p < (uint64_t)l_name + 4) return set_err(s, ORC_E_TRUNC, "reference %d truncated", i + 1);
    p += (uint64_t)l_name;
    s->ref_len[i] = rdi32(d + p);
    p += 4;
  }
  s->l_text = l_text;
  s->n_ref = n_ref < 0 ? 0 : n_ref;
  s->header_end = p;
  s->has_header = 1;
  return ORC_OK;
}

int orc_open(const uint8_t *f, uint64_t n, int check_crc, int want_header, orc_stream **out) {
  orc_stream *s = (orc_stream *)calloc(1, sizeof *s);
  if (!s) return ORC_E_NOMEM;
  *out = s;
  s->file_len = n;
  uint64_t cap = 1024;
  s->blk = (orc_block *)malloc(cap * sizeof(orc_block));
  uint64_t p = 0, u = 0;
  int rc;
  while (p < n) {
    if (s->nblk == cap) {
      cap *= 2;
      s->blk = (orc_block *)realloc(s->blk, cap * sizeof(orc_block));
    }
    orc_block *b = &s->blk[s->nblk];
    if ((rc = parse_block(s, f, n, p, b)) != ORC_OK) return rc;
    b->ustart = u;
    u += b->isize;
    p += b->csize;
    s->nblk++;
  }
  s->data = (uint8_t *)malloc(u ? u : 1);
  if (!s->data) return set_err(s, ORC_E_NOMEM, "oom");
  s->data_len = u;
  for (uint64_t k = 0; k < s->nblk; k++)
    if ((rc = inflate_block(s, f, &s->blk[k], s->data + s->blk[k].ustart, check_crc)) != ORC_OK) return rc;
  if (want_header) return parse_header(s);
  return ORC_OK;
}

void orc_close(orc_stream *s) {
  if (!s) return;
  free(s->ref_len);
  free(s->blk);
  free(s->data);
  free(s);
}
const char *orc_error(const orc_stream *s) { return s ? s->err : "null stream"; }
uint64_t orc_nblocks(const orc_stream *s) { return s->nblk; }
const orc_block *orc_blocks(const orc_stream *s) { return s->blk; }
const uint8_t *orc_data(const orc_stream *s) { return s->data; }
uint64_t orc_data_len(const orc_stream *s) { return s->data_len; }
int32_t orc_n_ref(const orc_stream *s) { return s->n_ref; }
int32_t orc_l_text(const orc_stream *s) { return s->l_text; }
uint64_t orc_header_end(const orc_stream *s) { return s->header_end; }
uint64_t orc_first_record_voff(const orc_stream *s) { return orc_voff_of(s, s->header_end); }

/* ------------------------------------------------------------------------ */
/* MurmurHash3 (util/MurmurHash3.java:32-102, fmix :173-180)                  */
/* ------------------------------------------------------------------------ */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

int64_t orc_murmurhash3(const uint8_t *key, uint64_t len64, int32_t seed) {
  const int32_t len = (int32_t)len64; /* Java byte[] length is an int */
  const int32_t nblocks = len / 16;
  uint64_t h1 = (uint64_t)(int64_t)seed, h2 = (uint64_t)(int64_t)seed; /* :41-42 sign-extended */
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int32_t i = 0; i < nblocks; i++) {
    uint64_t k1 = rd64(key + 16 * (uint64_t)i), k2 = rd64(key + 16 * (uint64_t)i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;                 /* :53 */
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;          /* :55 */
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;                 /* :57 */
    h2 = (h2 << 31) | (h1 >> 33); h2 += h1; h2 = h2 * 5 + 0x38495ab5; /* :59 quirk: h1>>>33 */
  }
  const uint8_t *t = key + 16 * (uint64_t)nblocks;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) { /* :68-88 */
  case 15: k2 ^= (uint64_t)t[14] << 48; /* fallthrough */
  case 14: k2 ^= (uint64_t)t[13] << 40; /* fallthrough */
  case 13: k2 ^= (uint64_t)t[12] << 32; /* fallthrough */
  case 12: k2 ^= (uint64_t)t[11] << 24; /* fallthrough */
  case 11: k2 ^= (uint64_t)t[10] << 16; /* fallthrough */
  case 10: k2 ^= (uint64_t)t[9] << 8;   /* fallthrough */
  case 9:  k2 ^= (uint64_t)t[8];
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;                 /* fallthrough */
  case 8: k1 ^= (uint64_t)t[7] << 56;   /* fallthrough */
  case 7: k1 ^= (uint64_t)t[6] << 48;   /* fallthrough */
  case 6: k1 ^= (uint64_t)t[5] << 40;   /* fallthrough */
  case 5: k1 ^= (uint64_t)t[4] << 32;   /* fallthrough */
  case 4: k1 ^= (uint64_t)t[3] << 24;   /* fallthrough */
  case 3: k1 ^= (uint64_t)t[2] << 16;   /* fallthrough */
  case 2: k1 ^= (uint64_t)t[1] << 8;    /* fallthrough */
  case 1: k1 ^= (uint64_t)t[0];
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;                 /* fallthrough */
  case 0: break;
  }
  h1 ^= (uint64_t)(int64_t)len; h2 ^= (uint64_t)(int64_t)len;         /* :90 */
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2;
  return (int64_t)h1;                                                  /* :101 */
}

/* BAMRecordReader.getKey (BAMRecordReader.java:81-121).  pos0 is the BAM pos
 * field; htsjdk's alignmentStart is pos0+1.  The unmapped branch hashes
 * getVariableBinaryRepresentation() = the block_size-32 bytes after the fixed
 * fields ([htsjdk] BAMRecord.mRestOfBinaryData). */
int64_t orc_get_key(int32_t ref_id, int32_t pos0, uint16_t flag, const uint8_t *var, uint32_t var_len) {
  int32_t start = (int32_t)((uint32_t)pos0 + 1u);
  if (!((flag & 4) || ref_id < 0 || start < 0)) /* :85 */
    return (int64_t)(((uint64_t)(int64_t)ref_id << 32) | (uint64_t)(int64_t)(int32_t)(start - 1)); /* :115,:120 */
  int32_t hash = (int32_t)orc_murmurhash3(var, var_len, 0);           /* :101 */
  return (int64_t)(((uint64_t)(int64_t)0x7fffffff << 32) | (uint64_t)(int64_t)hash); /* :110,:120 */
}

/* ------------------------------------------------------------------------ */
/* Span decode: BAMRecordReader.initialize (BAMRecordReader.java:151-154,181)*/
/* -> [htsjdk] BAMFileReader.getIterator(BAMFileSpan(Chunk(vStart,vEnd))):   */
/* seek(vStart); while getFilePointer() < vEnd: BAMRecordCodec.decode().     */
/* [htsjdk] BAMRecordCodec.decode: readInt(block_size) -> EOF (incl. partial */
/* int) ends the iteration; block_size < 32 -> SAMFormatException; short     */
/* record -> RuntimeEOFException; BAMRecord ctor resolves refID/next_refID   */
/* against the dictionary -> IllegalArgumentException if not in [-1,n_ref).  */
/* ------------------------------------------------------------------------ */
typedef struct {
  orc_records r;
  uint64_t cap;
} rec_buf;

static int rec_grow(rec_buf *b) {
  uint64_t c = b->cap ? b->cap * 2 : 4096;
#define GROW(field, T) do { void *q = realloc(b->r.field, c * sizeof(T)); if (!q) return ORC_E_NOMEM; b->r.field = (T *)q; } while (0)
  GROW(ref_id, int32_t); GROW(pos, int32_t); GROW(l_seq, int32_t); GROW(next_ref_id, int32_t);
  GROW(next_pos, int32_t); GROW(tlen, int32_t); GROW(l_read_name, uint8_t); GROW(mapq, uint8_t);
  GROW(bin, uint16_t); GROW(n_cigar, uint16_t); GROW(flag, uint16_t); GROW(key, int64_t);
  GROW(voff, uint64_t); GROW(offset, uint64_t); GROW(rest_len, uint32_t);
#undef GROW
  b->cap = c;
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* [htsjdk] SAMRecord.isValid(firstOnly) as BAMFileReader's iterator runs it */
/* on every record unless the stringency is SILENT; STRICT throws the first   */
/* error as a SAMFormatException, LENIENT only logs (but the lazy fields are  */
/* still decoded for the check, so a record whose read name / cigar / seq /   */
/* qual do not fit, or a cigar op code > 8, still fails).  Stringency comes   */
/* from hadoopbam.samheaderreader.validation-stringency                       */
/* (util/SAMHeaderReader.java:45-46, BAMRecordReader.java:142,192-194).       */
/* Restated rule list, parity unpinned by the reference:      */
/* no test of it asserts a validation error; test.bam (read under STRICT by   */
/* TestSplittingBAMIndexer) passes every rule.                                */
/* rec = the record's block_size field; returns 1 if invalid.                 */
/* ------------------------------------------------------------------------ */
static int32_t region_to_bin(int32_t beg, int32_t end) { /* GenomicIndexUtil.regionToBin */
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

/* aux lookup of a two-letter tag in t[0, len); *zlen = Z/H string length */
static int aux_has(const uint8_t *t, int64_t len, const char *tag, int64_t *zlen) {
  int64_t i = 0;
  while (i + 3 <= len) {
    const int hit = t[i] == (uint8_t)tag[0] && t[i + 1] == (uint8_t)tag[1];
    const uint8_t ty = t[i + 2];
    i += 3;
    int64_t sz;
    if (ty == 'A' || ty == 'c' || ty == 'C') sz = 1;
    else if (ty == 's' || ty == 'S') sz = 2;
    else if (ty == 'i' || ty == 'I' || ty == 'f') sz = 4;
    else if (ty == 'Z' || ty == 'H') {
      int64_t j = i;
      while (j < len && t[j]) j++;
      if (hit) *zlen = j - i;
      sz = j - i + 1;
    } else if (ty == 'B') {
      if (i + 5 > len) return 0;
      const uint8_t sub = t[i];
      const int64_t cnt = rdi32(t + i + 1);
      const int64_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
      if (cnt < 0) return 0;
      sz = 5 + cnt * es;
    } else {
      return 0;
    }
    if (hit) return 1;
    if (sz > len - i) return 0; /* a malformed aux block ends the lookup */
    i += sz;
  }
  return 0;
}

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };
static int op_real(uint32_t op) { return op == OP_M || op == OP_I || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X; }

int orc_record_invalid(const uint8_t *rec, int32_t bs, int32_t n_ref, const int32_t *ref_len, int strict) {
  const int32_t ref = rdi32(rec + 4), pos = rdi32(rec + 8);
  const uint32_t lrn = rec[12], mapq = rec[13], bin = rd16(rec + 14), ncig = rd16(rec + 16), flag = rd16(rec + 18);
  const int32_t lseq = rdi32(rec + 20), nref = rdi32(rec + 24), npos = rdi32(rec + 28);
  /* the lazily decoded fields must lie inside the record (BAMRecord offsets) */
  if (lrn < 1 || lseq < 0) return 1;
  if (32 + (int64_t)lrn + 4 * (int64_t)ncig + ((int64_t)lseq + 1) / 2 + (int64_t)lseq > (int64_t)bs) return 1;
  const uint8_t *cig = rec + 36 + lrn;
  for (uint32_t k = 0; k < ncig; k++)
    if ((rd32(cig + 4 * k) & 0xf) > 8) return 1; /* CigarOperator.binaryToEnum */
  if (!strict) return 0;
  const int paired = (flag & 0x1) != 0, unmapped = (flag & 0x4) != 0;
  if (!paired) { /* INVALID_FLAG_* of an unpaired read, INVALID_MATE_REF_INDEX */
    if (flag & 0x2 || flag & 0x8 || flag & 0x20 || flag & 0x40 || flag & 0x80) return 1;
    if (nref != -1) return 1;
  } else {
    /* isValidReferenceIndexAndPosition(mate): "*" <=> mate start 0 */
    if (nref == -1 && npos + 1 != 0) return 1;
    if (nref != -1 && npos + 1 == 0) return 1;
    if (nref != -1 && ref_len && (int64_t)npos + 1 > ref_len[nref]) return 1;
    if (nref == -1 && !(flag & 0x8)) return 1;       /* mapped mate needs a mate reference */
    if (!(flag & 0x40) && !(flag & 0x80)) return 1;  /* PAIRED_READ_NOT_MARKED_AS_FIRST_OR_SECOND */
  }
  if (unmapped) {
    if (flag & 0x100) return 1; /* INVALID_FLAG_NOT_PRIM_ALIGNMENT */
    if (flag & 0x800) return 1; /* INVALID_FLAG_SUPPLEMENTARY_ALIGNMENT */
    if (mapq != 0) return 1;    /* INVALID_MAPPING_QUALITY */
    /* htsjdk no longer rejects a cigar on an unmapped read ("now allowed,
       because there are current tools that do this"): test.bam has them */
  } else {
    if (ncig == 0) return 1;    /* INVALID_CIGAR: mapped read without cigar */
    if (n_ref == 0) return 1;   /* MISSING_SEQUENCE_DICTIONARY */
  }
  /* isValidReferenceIndexAndPosition(read) */
  if (ref == -1 && pos + 1 != 0) return 1;
  if (ref != -1 && pos + 1 == 0) return 1;
  if (ref != -1 && ref_len && (int64_t)pos + 1 > ref_len[ref]) return 1;
  /* Cigar.isValid + SAMUtils.validateCigar (mapped reads) */
  int64_t qlen = 0, rlen = 0;
  for (uint32_t k = 0; k < ncig; k++) {
    const uint32_t c = rd32(cig + 4 * k), op = c & 0xf, len = c >> 4;
    if (op == OP_M || op == OP_I || op == OP_S || op == OP_EQ || op == OP_X) qlen += len;
    if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rlen += len;
  }
  if (!unmapped) {
    int seen_real = 0;
    int64_t ref_at = (int64_t)pos + 1;
    for (uint32_t k = 0; k < ncig; k++) {
      const uint32_t c = rd32(cig + 4 * k), op = c & 0xf, len = c >> 4;
      if (len == 0) return 1; /* zero-length element */
      if (op == OP_H) {
        if (k != 0 && k != ncig - 1) return 1;
      } else if (op == OP_S) {
        if (k == 0 || k == ncig - 1) {
          /* soft clip at either end */
        } else if (k == 1) {
          const int three_with_h = ncig == 3 && (rd32(cig + 8) & 0xf) == OP_H;
          if (!three_with_h && (rd32(cig) & 0xf) != OP_H) return 1;
        } else if (k == ncig - 2) {
          if ((rd32(cig + 4 * (ncig - 1)) & 0xf) != OP_H) return 1;
        } else {
          return 1;
        }
      } else if (op == OP_P) {
        if (k != 0) {
          if (k == ncig - 1) return 1;
          if (!op_real(rd32(cig + 4 * (k - 1)) & 0xf) || !op_real(rd32(cig + 4 * (k + 1)) & 0xf)) return 1;
        }
      } else { /* real operator */
        seen_real = 1;
        if (op == OP_I || op == OP_D) { /* an M/N/=/X or P must separate two I or two D */
          for (uint32_t j = k + 1; j < ncig; j++) {
            const uint32_t nx = rd32(cig + 4 * j) & 0xf;
            if ((op_real(nx) && nx != OP_I && nx != OP_D) || nx == OP_P) break;
            if (nx == op) return 1;
          }
        }
      }
      if (op == OP_M || op == OP_EQ || op == OP_X) { /* alignment block inside the reference */
        if (ref >= 0 && ref_len && ref_at + len - 1 > ref_len[ref]) return 1;
      }
      if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) ref_at += len;
    }
    if (!seen_real) return 1;
  }
  { /* INVALID_INDEXING_BIN: computeIndexingBin() */
    const int32_t start0 = pos;
    int32_t end = unmapped ? 0 : (int32_t)((int64_t)pos + 1 + rlen - 1);
    if (end <= 0) end = start0 + 1;
    if ((uint32_t)region_to_bin(start0, end) != bin) return 1;
  }
  if (lseq != 0 && ncig != 0 && qlen != lseq) return 1; /* MISMATCH_CIGAR_SEQ_LENGTH */
  if (lseq == 0 && !(flag & 0x100)) { /* EMPTY_READ unless FZ, or non-empty CQ and CS */
    const uint8_t *aux = cig + 4 * ncig;
    const int64_t alen = (int64_t)bs - 32 - lrn - 4 * (int64_t)ncig;
    int64_t z = -1;
    if (!aux_has(aux, alen, "FZ", &z)) {
      int64_t cq = -1, cs = -1;
      const int hq = aux_has(aux, alen, "CQ", &cq), hs = aux_has(aux, alen, "CS", &cs);
      if (!hq || !hs || cq <= 0 || cs <= 0) return 1;
    }
  }
  return 0;
}

void orc_set_stringency(orc_stream *s, int stringency) { s->stringency = stringency; }

int orc_decode_span(orc_stream *s, uint64_t vstart, uint64_t vend, orc_records *out) {
  memset(out, 0, sizeof *out);
  rec_buf b;
  memset(&b, 0, sizeof b);
  int64_t sp = pos_of_voff(s, vstart);
  if (sp < 0) return set_err(s, ORC_E_IO, "Invalid file pointer: %llu", (unsigned long long)vstart);
  uint64_t p = (uint64_t)sp;
  const uint64_t end = s->data_len;
  const uint8_t *d = s->data;
  int rc = ORC_OK, first = 1;
  for (;; first = 0) {
    uint64_t v = orc_voff_of(s, p);
    if (v >= vend) break;                       /* chunk limit (span rule) */
    if (!first && dead_at(s, p)) break;         /* readInt -> EOF -> decode() == null */
    if (end - p < 4) break;                     /* partial int -> RuntimeEOF caught -> null */
    int32_t bs = rdi32(d + p);
    if (bs < 32) { rc = set_err(s, ORC_E_FORMAT, "Invalid record length: %d", bs); break; }
    if (dead_in_record(s, p, bs) || end - p - 4 < (uint64_t)bs) {
      rc = set_err(s, ORC_E_TRUNC, "Premature EOF in record at %llu", (unsigned long long)v);
      break;
    }
    const uint8_t *r = d + p;
    int32_t ref_id = rdi32(r + 4), next_ref = rdi32(r + 24);
    if (ref_id < -1 || ref_id >= s->n_ref) { rc = set_err(s, ORC_E_ARG, "Reference index %d not found in sequence dictionary.", ref_id); break; }
    if (next_ref < -1 || next_ref >= s->n_ref) { rc = set_err(s, ORC_E_ARG, "Reference index %d not found in sequence dictionary.", next_ref); break; }
    if (s->stringency != ORC_SILENT &&
        orc_record_invalid(r, bs, s->n_ref, s->ref_len, s->stringency == ORC_STRICT)) {
      rc = set_err(s, ORC_E_FORMAT, "SAMRecord.isValid failed at %llu", (unsigned long long)v);
      break;
    }
    if (b.r.n == b.cap && (rc = rec_grow(&b)) != ORC_OK) break;
    uint64_t i = b.r.n++;
    b.r.ref_id[i] = ref_id;
    b.r.pos[i] = rdi32(r + 8);
    b.r.l_read_name[i] = r[12];
    b.r.mapq[i] = r[13];
    b.r.bin[i] = rd16(r + 14);
    b.r.n_cigar[i] = rd16(r + 16);
    b.r.flag[i] = rd16(r + 18);
    b.r.l_seq[i] = rdi32(r + 20);
    b.r.next_ref_id[i] = next_ref;
    b.r.next_pos[i] = rdi32(r + 28);
    b.r.tlen[i] = rdi32(r + 32);
    b.r.voff[i] = v;
    b.r.offset[i] = p;
    b.r.rest_len[i] = (uint32_t)(bs - 32);
    b.r.key[i] = orc_get_key(ref_id, b.r.pos[i], b.r.flag[i], r + 36, (uint32_t)(bs - 32));
    p += 4 + (uint64_t)bs;
  }
  *out = b.r;
  return rc;
}

void orc_records_free(orc_records *r) {
  free(r->ref_id); free(r->pos); free(r->l_seq); free(r->next_ref_id); free(r->next_pos);
  free(r->tlen); free(r->l_read_name); free(r->mapq); free(r->bin); free(r->n_cigar);
  free(r->flag); free(r->key); free(r->voff); free(r->offset); free(r->rest_len);
  memset(r, 0, sizeof *r);
}
void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------------ */
/* SAMRecordWritable.write (SAMRecordWritable.java:55-64): [htsjdk]          */
/* BAMRecordCodec.encode of the BAMRecord BAMRecordReader hands out          */
/* (unmodified, lazily decoded).  Restated field by field:                   */
/*   blockSize = 32 + getReadNameLength()+1 + 4*cigarLen + (readLen+1)/2     */
/*             + readLen + getAttributesBinarySize(), the last being         */
/*             rest.length - (l_read_name + 4*n_cigar + (l_seq+1)/2 + l_seq) */
/*             ([htsjdk] BAMRecord; -1 = "stale" would re-encode the parsed  */
/*             attributes instead -- unreachable for records that decoded);  */
/*   indexBin  = refIndex >= 0 ? getIndexingBin() (the decoded bin) : 0;     */
/*   then refID, pos (=alignmentStart-1), l_read_name, mapq, bin, n_cigar,   */
/*   flag, l_seq, next_refID, next_pos, tlen, getVariableBinaryRepresentation*/
/*   (= the undecoded rest).  out may be NULL (size only); offs[i] = start   */
/*   of record i's encoding, offs[n] = total.                               */
/* ------------------------------------------------------------------------ */
static void put_le32(uint8_t *o, uint32_t v) {
  o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)(v >> 16); o[3] = (uint8_t)(v >> 24);
}
uint64_t orc_writable_encode(const uint8_t *data, const orc_records *r, uint8_t *out, uint64_t *offs) {
  uint64_t o = 0;
  for (uint64_t i = 0; i < r->n; i++) {
    const int64_t lrn = r->l_read_name[i], nc = r->n_cigar[i], ls = r->l_seq[i];
    const int64_t fixed_var = lrn + 4 * nc + (ls + 1) / 2 + ls;
    const int64_t attrs = (int64_t)r->rest_len[i] - fixed_var;
    const int32_t block_size = (int32_t)(32 + fixed_var + attrs);
    const uint16_t bin = r->ref_id[i] >= 0 ? r->bin[i] : 0;
    if (offs) offs[i] = o;
    if (out) {
      uint8_t *p = out + o;
      put_le32(p, (uint32_t)block_size);
      put_le32(p + 4, (uint32_t)r->ref_id[i]);
      put_le32(p + 8, (uint32_t)r->pos[i]);
      p[12] = r->l_read_name[i];
      p[13] = r->mapq[i];
      p[14] = (uint8_t)bin; p[15] = (uint8_t)(bin >> 8);
      p[16] = (uint8_t)r->n_cigar[i]; p[17] = (uint8_t)(r->n_cigar[i] >> 8);
      p[18] = (uint8_t)r->flag[i]; p[19] = (uint8_t)(r->flag[i] >> 8);
      put_le32(p + 20, (uint32_t)r->l_seq[i]);
      put_le32(p + 24, (uint32_t)r->next_ref_id[i]);
      put_le32(p + 28, (uint32_t)r->next_pos[i]);
      put_le32(p + 32, (uint32_t)r->tlen[i]);
      memcpy(p + 36, data + r->offset[i] + 36, r->rest_len[i]);
    }
    o += 4 + (uint64_t)(uint32_t)block_size;
  }
  if (offs) offs[r->n] = o;
  return o;
}

/* SAMRecordWritable.readFields (SAMRecordWritable.java:65-68): [htsjdk]     */
/* BAMRecordCodec.decode through LazyBAMRecordFactory with no header, once   */
/* per serialized value; value i is buf[offs[i], offs[i+1]), offs[n] = len.  */
/* readInt(block_size) hitting EOF makes decode() return null: reported as   */
/* ORC_E_TRUNC (a batch has no null record); block_size < 32 ->              */
/* SAMFormatException; a short rest -> RuntimeEOFException (ORC_E_TRUNC).    */
/* No dictionary check (null header).  offset = start of value i in buf;     */
/* voff = ~0 (a shuffled record has no file position).                       */
int orc_writable_decode(const uint8_t *buf, uint64_t len, const uint64_t *offs, uint64_t n, orc_records *out) {
  memset(out, 0, sizeof *out);
  rec_buf b;
  memset(&b, 0, sizeof b);
  int rc = ORC_OK;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t p = offs[i], e = i + 1 < n ? offs[i + 1] : len;
    if (e < p || e > len) { rc = ORC_E_ARG; break; }
    if (e - p < 4) { rc = ORC_E_TRUNC; break; }
    const uint8_t *r = buf + p;
    const int32_t bs = rdi32(r);
    if (bs < 32) { rc = ORC_E_FORMAT; break; }
    if (e - p - 4 < (uint64_t)bs) { rc = ORC_E_TRUNC; break; }
    if (b.r.n == b.cap && (rc = rec_grow(&b)) != ORC_OK) break;
    const uint64_t k = b.r.n++;
    b.r.ref_id[k] = rdi32(r + 4);
    b.r.pos[k] = rdi32(r + 8);
    b.r.l_read_name[k] = r[12];
    b.r.mapq[k] = r[13];
    b.r.bin[k] = rd16(r + 14);
    b.r.n_cigar[k] = rd16(r + 16);
    b.r.flag[k] = rd16(r + 18);
    b.r.l_seq[k] = rdi32(r + 20);
    b.r.next_ref_id[k] = rdi32(r + 24);
    b.r.next_pos[k] = rdi32(r + 28);
    b.r.tlen[k] = rdi32(r + 32);
    b.r.voff[k] = ~0ull;
    b.r.offset[k] = p;
    b.r.rest_len[k] = (uint32_t)(bs - 32);
    b.r.key[k] = orc_get_key(b.r.ref_id[k], b.r.pos[k], b.r.flag[k], r + 36, (uint32_t)(bs - 32));
  }
  *out = b.r;
  return rc;
}

/* ------------------------------------------------------------------------ */
/* SplittingBAMIndexer.index (SplittingBAMIndexer.java:248-290)              */
/* ------------------------------------------------------------------------ */
static void put_be64(uint8_t *o, uint64_t v) {
  for (int i = 0; i < 8; i++) o[i] = (uint8_t)(v >> (56 - 8 * i));
}

int orc_splitting_index(orc_stream *s, uint64_t file_size, int32_t g, uint8_t **out, uint64_t *out_len) {
  *out = NULL;
  *out_len = 0;
  if (!s->has_header) return set_err(s, ORC_E_IO, "no BAM header");
  uint64_t cap = 64, n = 0;
  uint64_t *v = (uint64_t *)malloc(cap * sizeof *v);
#define PUSH(x) do { if (n == cap) { cap *= 2; v = (uint64_t *)realloc(v, cap * sizeof *v); } v[n++] = (x); } while (0)
  const uint8_t *d = s->data;
  uint64_t p = s->header_end;                    /* skipToAlignmentList :292-328 */
  const uint64_t end = s->data_len;
  PUSH(orc_voff_of(s, p));                       /* :262-264 always write the first */
  int rc = ORC_OK;
  for (int32_t i = 0;;) {
    uint64_t ptr = orc_voff_of(s, p);            /* readAlignment :343 */
    uint64_t avail = end - p;
    if (avail == 0 || dead_at(s, p)) break;      /* read == 0 -> null :346 */
    if (avail < 4) { rc = set_err(s, ORC_E_IO, "Invalid alignment at virtual offset %#llx: less than 4 bytes long", (unsigned long long)orc_voff_of(s, end)); break; }
    int32_t skip = rdi32(d + p);
    p += 4;
    if (++i == g) { i = 0; PUSH(ptr); }          /* :273-277 */
    if (skip > 0) {                              /* fullySkip :355-368 */
      if ((uint64_t)skip > end - p || dead_at(s, p)) { rc = set_err(s, ORC_E_IO, "Skip failed"); break; }
      p += (uint64_t)skip;
    }
  }
  if (rc == ORC_OK) PUSH(file_size << 16);       /* :286 */
#undef PUSH
  if (rc != ORC_OK) { free(v); return rc; }
  uint8_t *o = (uint8_t *)malloc(n * 8);
  for (uint64_t k = 0; k < n; k++) put_be64(o + 8 * k, v[k]);
  free(v);
  *out = o;
  *out_len = n * 8;
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* BaseSplitGuesser.guessNextBGZFPos (BaseSplitGuesser.java:31-108) over a   */
/* ByteArraySeekableStream: IOUtils.readFully past the array end throws       */
/* (EOFException) -> null.                                                    */
/* ------------------------------------------------------------------------ */
#define BGZF_MAGIC 0x04088b1fu
#define BGZF_MAGIC_SUB 0x00024342u

int orc_guess_bgzf_pos(const uint8_t *a, uint64_t alen, int32_t p, int32_t end, int32_t *pos, int32_t *size) {
#define NEED(at, k) do { if ((int64_t)(at) < 0 || (uint64_t)(at) + (k) > alen) return 0; } while (0)
  for (;;) {
    for (;;) {
      NEED(p, 4);
      uint32_t nn = rd32(a + p);
      if (nn == BGZF_MAGIC) break;
      if ((nn >> 8) == ((BGZF_MAGIC << 8) >> 8)) ++p;
      else if ((nn >> 16) == ((BGZF_MAGIC << 16) >> 16)) p += 2;
      else p += 3;
      if (p >= end) return 0;
    }
    const int32_t p0 = p;
    p += 10;
    NEED(p, 2);
    int32_t xlen = rd16(a + p);
    p += 2;
    const int32_t subEnd = p + xlen;
    int found = 0;
    while (p < subEnd) {
      NEED(p, 4);
      uint32_t w = rd32(a + p);
      if (w != BGZF_MAGIC_SUB) {
        p += 4 + rd16(a + p + 2);
        continue;
      }
      NEED(p + 4, 2);
      int32_t bsize = rd16(a + p + 4);
      p += 6;
      while (p < subEnd) {
        NEED(p, 4);
        p += 4 + rd16(a + p + 2);
      }
      if (p != subEnd) break; /* cancel the guess */
      p += bsize - xlen - 19 + 4;
      NEED(p, 4);
      *pos = p0;
      *size = rdi32(a + p);
      found = 1;
      break;
    }
    if (found) return 1;
    p = p0 + 4;
  }
#undef NEED
}

/* BGZFSplitGuesser (util/BGZFSplitGuesser.java:64-167): same scan, accepts the
 * first candidate whose block inflates with CRC on.  in.read past the end
 * returns -1 and leaves the buffer unchanged (ByteArraySeekableStream). */
int64_t orc_guess_next_bgzf_block_start(const uint8_t *file, uint64_t flen, uint64_t beg, uint64_t end) {
  uint64_t want = end - beg;
  if (want > 2 * 0xffffu - 1) want = 2 * 0xffffu - 1;
  if (beg + want > flen) want = flen > beg ? flen - beg : 0;
  const uint8_t *a = file + beg;
  uint64_t alen = want;
  int32_t firstEnd = (int32_t)((end - beg) < 0xffff ? (end - beg) : 0xffff);
  uint8_t buf[8] = {0};
  for (int32_t pos = 0;;) {
    /* guessNextBGZFPos (:112-166) */
    int32_t p = pos, got = -1;
    for (;;) {
      for (;;) {
        for (int i = 0; i < 4; i++) if ((uint64_t)p + i < alen && p >= 0) buf[i] = a[p + i]; else if (i == 0 && (uint64_t)p >= alen) break;
        uint32_t nn = rd32(buf);
        if (nn == BGZF_MAGIC) break;
        if ((nn >> 8) == ((BGZF_MAGIC << 8) >> 8)) ++p;
        else if ((nn >> 16) == ((BGZF_MAGIC << 16) >> 16)) p += 2;
        else p += 3;
        if (p >= firstEnd) { got = -2; break; }
      }
      if (got == -2) break;
      int32_t p0 = p;
      p += 12;
      if ((uint64_t)p0 + 12 > alen) { got = -2; break; }
      int32_t xlen = rd16(a + p0 + 10), subEnd = p + xlen;
      while (p < subEnd) {
        if ((uint64_t)p + 4 > alen) break;
        if (rd32(a + p) != BGZF_MAGIC_SUB) { p += 4 + rd16(a + p + 2); continue; }
        got = p0;
        break;
      }
      if (got >= 0) break;
      p = p0 + 4;
    }
    if (got < 0) return (int64_t)end;
    pos = got;
    /* bgzf.seek(pos<<16): inflate the block with CRC check */
    orc_stream tmp;
    memset(&tmp, 0, sizeof tmp);
    orc_block b;
    int ok = parse_block(&tmp, a, alen, (uint64_t)pos, &b) == ORC_OK;
    if (ok) {
      uint8_t *dst = (uint8_t *)malloc(b.isize ? b.isize : 1);
      ok = inflate_block(&tmp, a, &b, dst, 1) == ORC_OK;
      free(dst);
    }
    if (!ok) { ++pos; continue; }
    return (int64_t)(beg + (uint64_t)pos);
  }
}

/* ------------------------------------------------------------------------ */
/* BAMSplitGuesser (BAMSplitGuesser.java:108-339).                            */
/* The guesser reads arr = file[beg, beg+min(end-beg, MAX_BYTES_READ)) and    */
/* runs an htsjdk BlockCompressedInputStream with CRC checks over it.        */
/* ------------------------------------------------------------------------ */
#define MAX_BYTES_READ (3 * 0xffff + 0xfffe)
#define SHORTEST_POSSIBLE_BAM_RECORD (4 * 9 + 1 + 1 + 1)

/* A BGZF reader over the guesser's array, restating the parts of [htsjdk]
 * BlockCompressedInputStream the guesser exercises. */
typedef struct {
  const uint8_t *a;
  uint64_t alen;
  /* cache of inflated blocks: index by array offset */
  uint64_t cur_coff;    /* block address of the current block */
  uint32_t cur_len;     /* compressed length */
  uint8_t *cur;         /* inflated data of the current block */
  uint32_t cur_isize;
  int has_cur;
  uint32_t off;         /* offset in current block */
  uint64_t next_coff;   /* stream offset of the next block */
  int eof;              /* last readBlock hit 0 header bytes */
} gz_reader;

enum { GZ_OK = 0, GZ_EOF = 1, GZ_ERR_TRUNC = 2, GZ_ERR_RUNTIMEIO = 3, GZ_ERR_FORMAT = 4, GZ_ERR_IO = 5 };

static void gz_free(gz_reader *g) { free(g->cur); g->cur = NULL; g->has_cur = 0; }

/* readBlock at stream offset c. */
static int gz_read_block(gz_reader *g, uint64_t c) {
  gz_free(g);
  g->eof = 0;
  if (c >= g->alen) { g->eof = 1; g->cur_coff = c; return GZ_EOF; } /* 0 header bytes */
  if (g->alen - c < 18) return GZ_ERR_IO;  /* "Incorrect header size" IOException */
  uint32_t total = (uint32_t)rd16(g->a + c + 16) + 1;
  if (total < 18 || total > 65536) return GZ_ERR_IO;
  if (c + total > g->alen) return GZ_ERR_TRUNC; /* FileTruncatedException */
  orc_stream tmp;
  memset(&tmp, 0, sizeof tmp);
  orc_block b;
  int rc = parse_block(&tmp, g->a, g->alen, c, &b);
  if (rc != ORC_OK) return rc == ORC_E_FORMAT ? GZ_ERR_FORMAT : GZ_ERR_IO;
  uint8_t *dst = (uint8_t *)malloc(b.isize ? b.isize : 1);
  rc = inflate_block(&tmp, g->a, &b, dst, 1);
  if (rc != ORC_OK) { free(dst); return rc == ORC_E_FORMAT ? GZ_ERR_FORMAT : GZ_ERR_RUNTIMEIO; }
  g->cur = dst;
  g->cur_isize = b.isize;
  g->cur_coff = c;
  g->cur_len = total;
  g->has_cur = 1;
  g->off = 0;
  g->next_coff = c + total;
  return GZ_OK;
}

/* seek(voff): [htsjdk] reuse the cached block if same address, else readBlock;
 * offset > length, or == length while not at EOF -> IOException. */
static int gz_seek(gz_reader *g, uint64_t voff) {
  uint64_t c = voff >> 16;
  uint32_t u = (uint32_t)(voff & 0xffff);
  if (!(g->has_cur && g->cur_coff == c)) {
    int rc = gz_read_block(g, c);
    if (rc == GZ_EOF) return GZ_ERR_IO;
    if (rc != GZ_OK) return rc;
  }
  if (u > g->cur_isize) return GZ_ERR_IO;
  if (u == g->cur_isize && g->next_coff < g->alen) return GZ_ERR_IO;
  g->off = u;
  return GZ_OK;
}

/* read up to n bytes; returns bytes read or negative error.  Empty block ->
 * EOF ([htsjdk] available()==0). */
static int64_t gz_read(gz_reader *g, uint8_t *dst, uint64_t n, int *err) {
  /* one [htsjdk] read(byte[],off,len) call: stops (partial) at an empty block,
   * returns -1 when nothing could be read */
  uint64_t got = 0;
  *err = GZ_OK;
  while (got < n) {
    if (!g->has_cur) break;
    if (g->off == g->cur_isize) {
      int rc = gz_read_block(g, g->next_coff);
      if (rc == GZ_EOF) break;
      if (rc != GZ_OK) { *err = rc; return -1; }
      if (g->cur_isize == 0) break; /* available()==0: EOF for this call */
      continue;
    }
    uint64_t k = g->cur_isize - g->off;
    if (k > n - got) k = n - got;
    memcpy(dst + got, g->cur + g->off, k);
    g->off += (uint32_t)k;
    got += k;
  }
  return (int64_t)got;
}

/* BinaryCodec.readBytes: loop of read calls; a call returning nothing -> EOF */
static int64_t gz_read_loop(gz_reader *g, uint8_t *dst, uint64_t n, int *err) {
  uint64_t got = 0;
  while (got < n) {
    int64_t r = gz_read(g, dst + got, n - got, err);
    if (r < 0) return -1;
    if (r == 0) break;
    got += (uint64_t)r;
  }
  return (int64_t)got;
}

static uint64_t gz_tell(const gz_reader *g) {
  if (!g->has_cur) return g->cur_coff << 16;
  if (g->off == g->cur_isize) return (g->cur_coff + g->cur_len) << 16;
  return (g->cur_coff << 16) | g->off;
}

/* IOUtils.readFully(bgzf, buf, 0, k): short read -> EOFException (IOException) */
static int gz_read_fully(gz_reader *g, uint8_t *dst, uint64_t k) {
  int err;
  int64_t r = gz_read_loop(g, dst, k, &err);
  if (r < 0) return err;
  if ((uint64_t)r < k) return GZ_ERR_IO;
  return GZ_OK;
}

/* guessNextBAMPos (BAMSplitGuesser.java:237-339). Returns up or -1; *fatal set
 * when a non-IOException escapes (propagates out of getSplits in Java). */
static int32_t guess_next_bam_pos(gz_reader *g, uint64_t cpVirt, int32_t up, int32_t cSize, int32_t n_ref, int *fatal) {
  uint8_t buf[8];
  *fatal = 0;
  up += 4;
  for (;;) {
    if (!(up + SHORTEST_POSSIBLE_BAM_RECORD - 4 < cSize)) return -1;
    int rc;
#define SEEKREAD(o, k)                                          \
  do {                                                          \
    rc = gz_seek(g, cpVirt | (uint64_t)(uint32_t)(o));          \
    if (rc == GZ_OK) rc = gz_read_fully(g, buf, (k));           \
    if (rc == GZ_ERR_IO || rc == GZ_EOF) return -1;             \
    if (rc != GZ_OK) {                                          \
      *fatal = 1;                                               \
      return -1;                                                \
    }                                                           \
  } while (0)
    SEEKREAD(up, 8);
    int32_t id = rdi32(buf), pos = rdi32(buf + 4);
    if (id < -1 || id > n_ref || pos < -1) { ++up; continue; }
    SEEKREAD(up + 20, 8);
    int32_t nid = rdi32(buf), npos = rdi32(buf + 4);
    if (nid < -1 || nid > n_ref || npos < -1) { ++up; continue; }
    int32_t nextUP = up + 1;
    up -= 4;
    SEEKREAD(up + 12, 4);
    int32_t nameLength = rdi32(buf) & 0xff;
    if (nameLength < 1) { up = nextUP; continue; }
    int32_t nullTerminator = up + 36 + nameLength - 1;
    if (nullTerminator >= cSize) { up = nextUP; continue; }
    SEEKREAD(nullTerminator, 1);
    if (buf[0] != 0) { up = nextUP; continue; }
    int32_t zeroMin = 4 * 8 + nameLength;
    SEEKREAD(up + 16, 8);
    zeroMin = (int32_t)((uint32_t)zeroMin + (uint32_t)((rdi32(buf) & 0xffff) * 4));
    int32_t l20 = rdi32(buf + 4);
    zeroMin = (int32_t)((uint32_t)zeroMin + (uint32_t)l20 + (uint32_t)((int32_t)((uint32_t)l20 + 1u) / 2));
    SEEKREAD(up, 4);
    if (rdi32(buf) < zeroMin) { up = nextUP; continue; }
    return up;
#undef SEEKREAD
  }
}

/* Structural restatement of [htsjdk] BAMRecordCodec.decode + setHeaderStrict +
 * BAMRecord.eagerDecode (SAMRecordHelper.java:7-10).  Returns:
 *   0 ok, 1 null (EOF at block_size), or an exception class. */
enum { DEC_OK = 0, DEC_NULL = 1, DEC_REJECT = 2, DEC_TRUNC = 3, DEC_EOF = 4, DEC_FATAL = 5 };

static int valid_aux(const uint8_t *t, int64_t len) {
  int64_t i = 0;
  while (i < len) {
    if (len - i < 3) return 0;
    uint8_t ty = t[i + 2];
    i += 3;
    int64_t sz;
    switch (ty) {
    case 'A': case 'c': case 'C': sz = 1; break;
    case 's': case 'S': sz = 2; break;
    case 'i': case 'I': case 'f': sz = 4; break;
    case 'Z': case 'H': {
      int64_t j = i;
      while (j < len && t[j]) j++;
      if (j >= len) return 0;
      sz = j - i + 1;
      break;
    }
    case 'B': {
      if (len - i < 5) return 0;
      uint8_t sub = t[i];
      int32_t cnt = rdi32(t + i + 1);
      int es;
      switch (sub) {
      case 'c': case 'C': es = 1; break;
      case 's': case 'S': es = 2; break;
      case 'i': case 'I': case 'f': es = 4; break;
      default: return 0;
      }
      if (cnt < 0) return 0;
      sz = 5 + (int64_t)cnt * es;
      break;
    }
    default: return 0;
    }
    if (len - i < sz) return 0;
    i += sz;
  }
  return 1;
}

static int decode_verify(gz_reader *g, int32_t n_ref) {
  uint8_t hdr[36];
  int err;
  int64_t r = gz_read_loop(g, hdr, 4, &err);
  if (r < 0) return err == GZ_ERR_TRUNC ? DEC_TRUNC : DEC_REJECT; /* FileTruncated / RuntimeIO+Format */
  if (r < 4) return DEC_NULL;                                       /* RuntimeEOF caught in decode */
  int32_t bs = rdi32(hdr);
  if (bs < 32) return DEC_REJECT;                                   /* SAMFormatException */
  uint8_t *rec = (uint8_t *)malloc((size_t)bs);
  r = gz_read_loop(g, rec, (uint64_t)bs, &err);
  if (r < 0) { free(rec); return err == GZ_ERR_TRUNC ? DEC_TRUNC : DEC_REJECT; }
  if (r < bs) { free(rec); return DEC_EOF; }                        /* RuntimeEOFException */
  int32_t ref = rdi32(rec), nref = rdi32(rec + 20);
  int ok = 1;
  if (ref < -1 || ref >= n_ref || nref < -1 || nref >= n_ref) ok = 0; /* setHeaderStrict */
  int32_t lrn = rec[8], ncig = rd16(rec + 12), lseq = rdi32(rec + 16);
  int64_t rest = bs - 32;
  const uint8_t *v = rec + 32;
  if (ok && lrn < 1) ok = 0;                                        /* name length-1 < 0 */
  if (ok && lrn - 1 > rest) ok = 0;
  if (ok && (int64_t)lrn + 4 * (int64_t)ncig > rest) ok = 0;        /* cigar buffer */
  if (ok) for (int32_t k = 0; k < ncig; k++) if ((rd32(v + lrn + 4 * k) & 0xf) > 8) { ok = 0; break; }
  int64_t seqoff = (int64_t)lrn + 4 * (int64_t)ncig;
  if (ok && lseq < 0) ok = 0;
  if (ok && lseq > 0 && seqoff + ((int64_t)lseq + 1) / 2 > rest) ok = 0;
  int64_t tagoff = seqoff + ((int64_t)lseq + 1) / 2 + lseq;
  if (ok && tagoff > rest) ok = 0;
  if (ok && !valid_aux(v + tagoff, rest - tagoff)) ok = 0;
  free(rec);
  return ok ? DEC_OK : DEC_REJECT;
}

int orc_guess_record_start(orc_stream *s, const uint8_t *file, uint64_t flen, uint64_t beg, uint64_t end, uint64_t *out) {
  return orc_guess_record_start_hdr(s, file, flen, s->n_ref, beg, end, out);
}

/* BAMSplitGuesser(ss, headerStream, conf) (BAMSplitGuesser.java:93-103): the
 * record checks bound refIDs by the header stream's dictionary (n_ref), the
 * first record of beg == 0 still comes from the data (:115-123) */
int orc_guess_record_start_hdr(orc_stream *s, const uint8_t *file, uint64_t flen, int32_t n_ref, uint64_t beg,
                               uint64_t end, uint64_t *out) {
  if (beg == 0) { /* :115-123 header parse -> first record voff */
    *out = orc_first_record_voff(s);
    return ORC_OK;
  }
  uint64_t want = end - beg;
  if (want > MAX_BYTES_READ) want = MAX_BYTES_READ;
  if (beg + want > flen) want = flen > beg ? flen - beg : 0;
  gz_reader g;
  memset(&g, 0, sizeof g);
  g.a = file + beg;
  g.alen = want;
  const int32_t firstEnd = (int32_t)((end - beg) < 0xffff ? (end - beg) : 0xffff);
  for (int32_t cp = 0;; ++cp) {
    int32_t ppos, psize;
    if (!orc_guess_bgzf_pos(g.a, g.alen, cp, firstEnd, &ppos, &psize)) { gz_free(&g); *out = end; return ORC_OK; }
    const int32_t cp0 = cp = ppos;
    const uint64_t cp0Virt = (uint64_t)cp0 << 16;
    if (gz_seek(&g, cp0Virt) != GZ_OK) continue; /* catch Throwable */
    for (int32_t up = 0;; ++up) {
      int fatal;
      const int32_t up0 = up = guess_next_bam_pos(&g, cp0Virt, up, psize, n_ref, &fatal);
      if (fatal) { gz_free(&g); return set_err(s, ORC_E_FORMAT, "exception escaped guessNextBAMPos"); }
      if (up0 < 0) break;
      if (gz_seek(&g, cp0Virt | (uint64_t)up0) != GZ_OK) continue;
      int decodedAny = 0, accept = 1;
      int b = 0;
      uint64_t prevCP = (uint64_t)cp0;
      while (b < 3) {
        int dr = decode_verify(&g, n_ref);
        if (dr == DEC_NULL) break;
        if (dr == DEC_REJECT) { accept = 0; break; }
        if (dr == DEC_TRUNC || dr == DEC_EOF) {  /* FileTruncated / RuntimeEOF */
          int in_eof = 1; /* the array stream is exhausted once the reader hit its end */
          if (!decodedAny && in_eof) accept = 0;
          break;
        }
        decodedAny = 1;
        uint64_t cp2 = gz_tell(&g) >> 16;
        if (cp2 != prevCP) { prevCP = cp2; ++b; }
      }
      if (accept && b < 3 && !decodedAny) accept = 0;
      if (!accept) continue;
      gz_free(&g);
      *out = ((beg + (uint64_t)cp0) << 16) | (uint64_t)up0;
      return ORC_OK;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Split planning (BAMInputFormat.java:264-318 addIndexedSplits,             */
/* 469-530 addProbabilisticSplits) for the FileSplits of ONE file.           */
/* SplittingBAMIndex.readIndex :52-72, prevAlignment (floor) :78-80,          */
/* nextAlignment (strictly higher) :81-83.                                   */
/* ------------------------------------------------------------------------ */
static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

int orc_get_splits(orc_stream *s, const uint8_t *file, uint64_t flen, const uint64_t *starts, const uint64_t *lengths,
                   uint64_t n, const uint8_t *sbi, uint64_t sbi_len, uint64_t *vs, uint64_t *ve, uint64_t *nout) {
  *nout = 0;
  int use_index = sbi != NULL;
  uint64_t *idx = NULL, ni = 0;
  if (use_index) {
    idx = (uint64_t *)malloc((sbi_len / 8 + 1) * sizeof *idx);
    int64_t prev = -1;
    for (uint64_t k = 0; k + 8 <= sbi_len; k += 8) {
      uint64_t cur = 0;
      for (int i = 0; i < 8; i++) cur = (cur << 8) | sbi[k + i];
      if (prev > (int64_t)cur) { free(idx); return set_err(s, ORC_E_IO, "Invalid splitting BAM index; offsets not in order"); }
      prev = (int64_t)cur;
      idx[ni++] = cur;
    }
    if (ni < 1) { free(idx); return set_err(s, ORC_E_IO, "Invalid splitting BAM index: should contain at least the file size"); }
    qsort(idx, ni, sizeof *idx, cmp_u64);
    uint64_t m = 0; /* TreeSet de-dup */
    for (uint64_t k = 0; k < ni; k++) if (m == 0 || idx[m - 1] != idx[k]) idx[m++] = idx[k];
    ni = m;
    if (ni == 1) { free(idx); return ORC_OK; } /* :280-282 no alignments */
    int good = 1;
    for (uint64_t j = 0; j < n && good; j++) {
      uint64_t start = starts[j], e = start + lengths[j];
      /* nextAlignment(start): strictly higher than start<<16 */
      uint64_t key = start << 16, bs = 0, be = 0;
      int hs = 0, he = 0;
      for (uint64_t k = 0; k < ni; k++) if (idx[k] > key) { bs = idx[k]; hs = 1; break; }
      if (j == n - 1) { /* prevAlignment(end) | 0xffff */
        uint64_t ke = e << 16;
        for (uint64_t k = ni; k-- > 0;) if (idx[k] <= ke) { be = idx[k] | 0xffff; he = 1; break; }
      } else {
        uint64_t ke = e << 16;
        for (uint64_t k = 0; k < ni; k++) if (idx[k] > ke) { be = idx[k]; he = 1; break; }
      }
      if (!hs || !he) { good = 0; break; }
      vs[*nout] = bs;
      ve[*nout] = be;
      (*nout)++;
    }
    free(idx);
    if (good) return ORC_OK;
    *nout = 0; /* :305-308 bad index -> probabilistic */
  }
  int64_t prev = -1;
  for (uint64_t j = 0; j < n; j++) {
    uint64_t beg = starts[j], e = beg + lengths[j], ab;
    int rc = orc_guess_record_start(s, file, flen, beg, e, &ab);
    if (rc != ORC_OK) return rc;
    uint64_t ae = (e << 16) | 0xffff;
    if (ab == e) {
      if (prev < 0) return set_err(s, ORC_E_IO, "no reads in first split: bad BAM file or tiny split size?");
      ve[prev] = ae;
    } else {
      vs[*nout] = ab;
      ve[*nout] = ae;
      prev = (int64_t)(*nout)++;
    }
  }
  return ORC_OK;
}
