/*
 * gen_synth_bam.c -- deterministic synthetic BAM writer (bench / test INPUT
 * generator; it compresses with zlib and is never part of the read path).
 *
 * Models:
 *   mode 0  "C2": paired-end 150 bp, coordinate-sorted over 25 hg19-like
 *           contigs at ~30x local coverage; 98 % mapped (1-3 CIGAR ops),
 *           1.5 % unmapped-placed (mate's refID/pos), 0.5 % unplaced at the end;
 *           read names SYN-HS2000:<lane>:FC706VJ:<swath>:<tile>:<x>:<y>; Illumina-like per-cycle qualities;
 *           aux NM:i MD:Z AS:i XS:i RG:Z.
 *   mode 1  "C4": ONT-like long reads, 10-50 kb (log-normal, median 20 kb),
 *           Q 5-30, CIGARs of 100s-1000s of ops, MM:Z + ML:B:C, 10 % unmapped.
 *   mode 2  "C3": mode 0 with the qualities binned to the 8 levels of
 *           Illumina's quality binning (2, 6, 15, 22, 27, 33, 37, 40), as
 *           30x WGS BAMs from binned-quality instruments hold them: ~100 B
 *           per record compressed, so ~600 M reads are ~60 GB, as BASELINE
 *           config 3 names it (mode 0's unbinned qualities: ~141 B).
 * BGZF framing as htsjdk/htslib write it (1f8b0804 00000000 00ff 0600 4243 0200
 * BSIZE); raw DEFLATE at a chosen level/strategy; payload cut every
 * `block_payload` bytes regardless of record boundaries; optional EOF block.
 * Record i is a pure function of (seed, i): generation and compression run in
 * parallel threads.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

typedef struct {
  uint64_t n_records;
  int32_t mode;           /* 0 short PE, 1 long reads, 2 short PE with binned qualities */
  int32_t level;          /* zlib level (htsjdk default 5) */
  int32_t strategy;       /* Z_DEFAULT_STRATEGY(0) Z_FILTERED(1) Z_HUFFMAN_ONLY(2) Z_RLE(3) Z_FIXED(4) */
  int32_t block_payload;  /* uncompressed bytes per BGZF block (<= 65280 for stored safety) */
  int32_t threads;
  int32_t eof_block;      /* append the 28-byte EOF marker */
  int32_t all_unmapped;   /* every record unmapped-placed (flag 4), like test.bam */
  uint64_t seed;
} gen_params;

static const char *kContig[25] = {"chr1",  "chr2",  "chr3",  "chr4",  "chr5",  "chr6",  "chr7",
                                  "chr8",  "chr9",  "chr10", "chr11", "chr12", "chr13", "chr14",
                                  "chr15", "chr16", "chr17", "chr18", "chr19", "chr20", "chr21",
                                  "chr22", "chrX",  "chrY",  "chrM"};
static const int32_t kContigLen[25] = {249250621, 243199373, 198022430, 191154276, 180915260,
                                       171115067, 159138663, 146364022, 141213431, 135534747,
                                       135006516, 133851895, 115169878, 107349540, 102531392,
                                       90354753,  81195210,  78077248,  59128983,  63025520,
                                       48129895,  51304566,  155270560, 59373566,  16571};

static inline uint64_t splitmix(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static inline uint64_t hash2(uint64_t a, uint64_t b) {
  uint64_t s = a * 0x9e3779b97f4a7c15ULL ^ b;
  return splitmix(&s);
}
/* reference base at genomic coordinate g of contig c (0..3 = ACGT) */
static inline int ref_base(int c, uint64_t g) { return (int)(hash2(0x5eed0000ULL + (uint64_t)c, g >> 5) >> (2 * (g & 31))) & 3; }

typedef struct {
  const gen_params *p;
  uint64_t n_mapped, n_unplaced_start;
  uint64_t span;  /* genomic span covered by mapped reads (bp) */
} model;

static void put16(uint8_t *o, uint16_t v) { o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); }
static void put32(uint8_t *o, uint32_t v) { o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)(v >> 16); o[3] = (uint8_t)(v >> 24); }

/* UCSC binning (reg2bin) */
static int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

/* position of mapped record i: genome walk at 30x local coverage; a read
 * (<= 50 kb of reference for long reads) never runs off its contig */
static void locus(const model *m, uint64_t i, int *ref, int32_t *pos) {
  /* start of read i: an even walk plus jitter below one step, so starts
   * stay sorted but their spacing (and the seq nibble phase) varies */
  const uint64_t step = m->span / (m->n_mapped ? m->n_mapped : 1);
  uint64_t g = (i * m->span) / (m->n_mapped ? m->n_mapped : 1) + (step > 1 ? hash2(0x10c05ULL, i) % step : 0);
  int c = 0;
  while (c < 24 && g >= (uint64_t)kContigLen[c]) { g -= (uint64_t)kContigLen[c]; ++c; }
  /* short reads: the first mate's mate starts 200 bp on, and a mate start
   * must lie inside the contig (STRICT: 1-based start <= length), so 201 */
  const uint64_t room = m->p->mode == 1 ? 60000 : 201;
  if (g + room > (uint64_t)kContigLen[c]) g = kContigLen[c] > (int32_t)room ? (uint64_t)kContigLen[c] - room : 0;
  *ref = c;
  *pos = (int32_t)g;
}

/* Writes record i into o (if o != NULL); returns its total size incl. block_size. */
static uint32_t make_record(const model *m, uint64_t i, uint8_t *o) {
  const gen_params *p = m->p;
  uint64_t s = hash2(p->seed, i);
  uint8_t buf[64];
  int ref = -1, mref = -1;
  int32_t pos = -1, mpos = -1, tlen = 0;
  uint16_t flag;
  uint8_t mapq;
  int unmapped = 0, unplaced = 0;
  int l_seq;
  uint32_t ncig = 0;
  uint32_t cig[4096];
  if (i >= m->n_unplaced_start) {
    unplaced = 1;
    unmapped = 1;
  } else {
    locus(m, i, &ref, &pos);
    uint64_t r = splitmix(&s) % 1000;
    if (p->all_unmapped || r < (p->mode == 1 ? 100u : 15u)) unmapped = 1;
  }
  /* read length */
  if (p->mode != 1) {
    l_seq = 150;
  } else {
    /* log-normal-ish: median 20 kb, clipped 10-50 kb */
    double u1 = ((splitmix(&s) >> 11) + 0.5) / 9007199254740992.0, u2 = ((splitmix(&s) >> 11) + 0.5) / 9007199254740992.0;
    double z = 0;
    { /* Box-Muller without libm: approximate with sum of uniforms */
      z = (u1 + u2 + ((splitmix(&s) >> 11) / 9007199254740992.0) - 1.5) * 2.0;
    }
    double len = 20000.0 * (1.0 + 0.45 * z + 0.1 * z * z);
    if (len < 10000) len = 10000;
    if (len > 50000) len = 50000;
    l_seq = (int)len;
  }
  const uint64_t pair = i >> 1;
  const int mate = (int)(i & 1);
  if (unplaced) {
    flag = 0x1 | 0x4 | 0x8 | (mate ? 0x80 : 0x40);
    mapq = 0;
    ref = mref = -1;
    pos = mpos = -1;
  } else if (unmapped) {
    flag = (p->mode != 1 ? (0x1 | (mate ? 0x80 : 0x40)) : 0) | 0x4;
    mapq = 0;
    mref = p->mode != 1 ? ref : -1;
    mpos = p->mode != 1 ? pos : -1;
    if (p->mode == 1) { ref = -1; pos = -1; }
  } else {
    mapq = (uint8_t)(20 + splitmix(&s) % 41);
    if (p->mode != 1) {
      flag = 0x1 | 0x2 | (mate ? 0x80 : 0x40) | (mate ? 0x10 : 0x20);
      mref = ref;
      mpos = pos + (mate ? -200 : 200);
      if (mpos < 0) mpos = 0;
      tlen = mate ? -350 : 350;
      /* 1-3 ops summing to l_seq query bases */
      uint64_t k = splitmix(&s) % 10;
      if (k < 6) { cig[ncig++] = (uint32_t)l_seq << 4 | 0; }
      else if (k < 8) { int sc = 1 + (int)(splitmix(&s) % 20); cig[ncig++] = (uint32_t)sc << 4 | 4; cig[ncig++] = (uint32_t)(l_seq - sc) << 4 | 0; }
      else { int a = 30 + (int)(splitmix(&s) % 90), d = 1 + (int)(splitmix(&s) % 3); cig[ncig++] = (uint32_t)a << 4 | 0; cig[ncig++] = (uint32_t)d << 4 | 1; cig[ncig++] = (uint32_t)(l_seq - a - d) << 4 | 0; }
    } else {
      flag = (splitmix(&s) & 1) ? 0x10 : 0;
      mref = -1;
      mpos = -1;
      /* many ops: alternating M / I / D every ~20-200 bases */
      int left = l_seq;
      while (left > 0 && ncig < 4000) {
        int mlen = 20 + (int)(splitmix(&s) % 180);
        if (mlen > left) mlen = left;
        cig[ncig++] = (uint32_t)mlen << 4 | 0;
        left -= mlen;
        if (left <= 0) break;
        uint64_t t = splitmix(&s) % 3;
        if (t == 0) { int il = 1 + (int)(splitmix(&s) % 4); if (il > left) il = left; cig[ncig++] = (uint32_t)il << 4 | 1; left -= il; }
        else if (t == 1) { cig[ncig++] = (uint32_t)(1 + splitmix(&s) % 4) << 4 | 2; }
      }
      if (left > 0) cig[ncig++] = (uint32_t)left << 4 | 4;
    }
  }
  /* read name */
  char name[64];
  uint64_t ns = hash2(p->seed ^ 0xabcdefULL, pair);
  int nl = snprintf(name, sizeof name, "SYN-HS2000:%u:FC706VJ:%u:%u:%u:%u", (unsigned)(1 + ns % 8),
                    (unsigned)(1 + (ns >> 3) % 8), (unsigned)(1101 + (ns >> 6) % 68), (unsigned)((ns >> 16) % 21000),
                    (unsigned)((ns >> 32) % 200000));
  const int l_read_name = nl + 1;
  /* aux */
  char md[64];
  int nm = (int)(splitmix(&s) % 4);
  int mdl = nm ? snprintf(md, sizeof md, "%dA%dC%d", l_seq / 2, 3, l_seq - l_seq / 2 - 5) : snprintf(md, sizeof md, "%d", l_seq);
  int aux_len = 0;
  if (p->mode != 1) {
    aux_len += 3 + 1;                 /* NM:C */
    aux_len += 3 + mdl + 1;           /* MD:Z */
    aux_len += 3 + 1 + 3 + 1;         /* AS:C XS:C */
    aux_len += 3 + 8;                 /* RG:Z:SYN.1.1 */
  } else {
    aux_len += 3 + 8;                 /* RG */
    aux_len += 3 + 9 + 1;             /* MM:Z:C+m?,... short */
    aux_len += 3 + 1 + 4 + l_seq / 4; /* ML:B:C */
  }
  const int32_t bs = 32 + l_read_name + 4 * (int32_t)ncig + l_seq + (l_seq + 1) / 2 + aux_len;
  const uint32_t total = 4 + (uint32_t)bs;
  if (!o) return total;
  /* ---- write ---- */
  int end = pos;
  for (uint32_t k = 0; k < ncig; ++k) { int op = cig[k] & 0xf; if (op == 0 || op == 2) end += (int)(cig[k] >> 4); }
  /* htsjdk computeIndexingBin: reg2bin(alignmentStart-1, alignmentEnd), a
   * one-base span when the read is unmapped (unplaced: reg2bin(-1, 0) = 4680) */
  int bin = pos < 0 ? 4680 : reg2bin(pos, (!unmapped && end > pos) ? end : pos + 1);
  put32(o, (uint32_t)bs);
  put32(o + 4, (uint32_t)ref);
  put32(o + 8, (uint32_t)pos);
  o[12] = (uint8_t)l_read_name;
  o[13] = mapq;
  put16(o + 14, (uint16_t)bin);
  put16(o + 16, (uint16_t)ncig);
  put16(o + 18, flag);
  put32(o + 20, (uint32_t)l_seq);
  put32(o + 24, (uint32_t)mref);
  put32(o + 28, (uint32_t)mpos);
  put32(o + 32, (uint32_t)tlen);
  uint8_t *w = o + 36;
  memcpy(w, name, (size_t)nl);
  w[nl] = 0;
  w += l_read_name;
  for (uint32_t k = 0; k < ncig; ++k, w += 4) put32(w, cig[k]);
  /* seq: copy of the pseudo-reference with a few mismatches (4-bit =ACMGRSVTWYHKDBN: A=1 C=2 G=4 T=8) */
  static const uint8_t code[4] = {1, 2, 4, 8};
  uint64_t ms = hash2(p->seed ^ 0x77ULL, i);
  for (int k = 0; k < l_seq; k += 2) {
    uint8_t hi, lo;
    int c0 = ref < 0 ? (int)(splitmix(&ms) & 3) : ref_base(ref, (uint64_t)(pos + k));
    int c1 = ref < 0 ? (int)(splitmix(&ms) & 3) : ref_base(ref, (uint64_t)(pos + k + 1));
    {  /* ~1.5 % substitutions on either base of the pair (errors + SNVs) */
      const uint64_t e = splitmix(&ms);
      if ((e & 63) == 0) c0 = (c0 + 1 + (int)((e >> 8) % 3)) & 3;
      if (((e >> 16) & 63) == 0) c1 = (c1 + 1 + (int)((e >> 24) % 3)) & 3;
    }
    hi = code[c0];
    lo = (k + 1 < l_seq) ? code[c1] : 0;
    *w++ = (uint8_t)(hi << 4 | lo);
  }
  /* qual: Illumina-like per-cycle model for short reads -- mean 37 falling
   * to ~30 over the read, per-base noise ~N(0, 4.3) (Q2..Q41), 2 % isolated
   * low-quality calls and, in 8 % of reads, a Q2 tail (the Illumina read
   * segment indicator) -- about 3.9 bits per quality after DEFLATE, which puts
   * C2 at ~1.5 GB compressed as SURVEY 8d asks; ONT-like random walk Q5..30
   * for long reads */
  if (p->mode != 1) {
    uint64_t tr = splitmix(&ms);
    const int tail = (tr % 100) < 8 ? l_seq - 5 - (int)((tr >> 8) % 40) : l_seq;
    for (int k = 0; k < l_seq; ++k) {
      uint64_t r = splitmix(&ms);
      const int sum = (int)(r & 255) + (int)((r >> 8) & 255) + (int)((r >> 16) & 255) + (int)((r >> 24) & 255);
      int q = 36 - k / 20 + (sum - 510) / 30;
      if (((r >> 32) & 63) == 0) q = 2 + (int)((r >> 40) % 12);
      if (k >= tail) q = 2;
      if (q > 41) q = 41;
      if (q < 2) q = 2;
      if (p->mode == 2) q = q < 3 ? 2 : q < 10 ? 6 : q < 20 ? 15 : q < 25 ? 22 : q < 30 ? 27 : q < 35 ? 33 : q < 40 ? 37 : 40;
      *w++ = (uint8_t)q;
    }
  } else {
    int q = 18;
    for (int k = 0; k < l_seq; ++k) {
      uint64_t r = splitmix(&ms);
      int d = (int)(r % 7) - 3;
      q += d / 2;
      if (q > 30) q = 30;
      if (q < 5) q = 5;
      *w++ = (uint8_t)q;
    }
  }
  if (p->mode != 1) {
    memcpy(w, "NMC", 3); w[3] = (uint8_t)nm; w += 4;
    memcpy(w, "MDZ", 3); memcpy(w + 3, md, (size_t)mdl); w[3 + mdl] = 0; w += 3 + mdl + 1;
    memcpy(w, "ASC", 3); w[3] = (uint8_t)(l_seq - 5 * nm); w += 4;
    memcpy(w, "XSC", 3); w[3] = (uint8_t)(l_seq / 2); w += 4;
    memcpy(w, "RGZ", 3); memcpy(w + 3, "SYN.1.1", 8); w += 11;
  } else {
    memcpy(w, "RGZ", 3); memcpy(w + 3, "SYN.1.1", 8); w += 11;
    memcpy(w, "MMZ", 3); memcpy(w + 3, "C+m?,1,0;", 10); w += 13;
    memcpy(w, "MLB", 3); w[3] = 'C'; put32(w + 4, (uint32_t)(l_seq / 4)); w += 8;
    for (int k = 0; k < l_seq / 4; ++k) *w++ = (uint8_t)(splitmix(&ms) & 255);
  }
  if ((uint32_t)(w - o) != total) { fprintf(stderr, "gen: size mismatch %u vs %u\n", (unsigned)(w - o), total); abort(); }
  return total;
}

static size_t make_header(uint8_t *o) {
  char text[4096];
  int tl = snprintf(text, sizeof text, "@HD\tVN:1.6\tSO:coordinate\n");
  for (int c = 0; c < 25; ++c) tl += snprintf(text + tl, sizeof text - (size_t)tl, "@SQ\tSN:%s\tLN:%d\n", kContig[c], kContigLen[c]);
  tl += snprintf(text + tl, sizeof text - (size_t)tl, "@RG\tID:SYN.1.1\tSM:synthetic\tPL:ILLUMINA\n");
  size_t n = 0;
  if (o) { memcpy(o, "BAM\1", 4); put32(o + 4, (uint32_t)tl); memcpy(o + 8, text, (size_t)tl); }
  n = 8 + (size_t)tl;
  if (o) put32(o + n, 25);
  n += 4;
  for (int c = 0; c < 25; ++c) {
    int ln = (int)strlen(kContig[c]) + 1;
    if (o) { put32(o + n, (uint32_t)ln); memcpy(o + n + 4, kContig[c], (size_t)ln); put32(o + n + 4 + ln, (uint32_t)kContigLen[c]); }
    n += 4 + (size_t)ln + 4;
  }
  return n;
}

typedef struct {
  const model *m;
  uint64_t lo, hi;          /* record range */
  uint64_t base;            /* first record of the segment: sizes / offs index i - base */
  uint32_t *sizes;
  uint64_t *offs;
  uint8_t *u;
  int phase;
  /* compression */
  const uint8_t *src;
  uint64_t usz;
  uint64_t blk_lo, blk_hi;
  uint8_t **cblk;
  uint32_t *clen;
  int err;
} job;

static void *worker(void *arg) {
  job *j = (job *)arg;
  const gen_params *p = j->m->p;
  if (j->phase == 0) {
    for (uint64_t i = j->lo; i < j->hi; ++i) j->sizes[i - j->base] = make_record(j->m, i, NULL);
  } else if (j->phase == 1) {
    for (uint64_t i = j->lo; i < j->hi; ++i) make_record(j->m, i, j->u + j->offs[i - j->base]);
  } else {
    z_stream z;
    for (uint64_t b = j->blk_lo; b < j->blk_hi; ++b) {
      uint64_t a = b * (uint64_t)p->block_payload;
      uint64_t e = a + (uint64_t)p->block_payload;
      if (e > j->usz) e = j->usz;
      uint32_t in = (uint32_t)(e - a);
      uint8_t *o = (uint8_t *)malloc(65536 + 1024);
      memset(&z, 0, sizeof z);
      if (deflateInit2(&z, p->level, Z_DEFLATED, -15, 8, p->strategy) != Z_OK) { j->err = 1; free(o); return NULL; }
      z.next_in = (Bytef *)(j->src + a);
      z.avail_in = in;
      z.next_out = o + 18;
      z.avail_out = 65536 - 26;
      int rc = deflate(&z, Z_FINISH);
      uint32_t cl = (uint32_t)(65536 - 26 - z.avail_out);
      deflateEnd(&z);
      if (rc != Z_STREAM_END) { j->err = 2; free(o); return NULL; }
      uint32_t total = 18 + cl + 8;
      static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
      memcpy(o, hdr, 16);
      put16(o + 16, (uint16_t)(total - 1));
      put32(o + 18 + cl, (uint32_t)crc32(0L, j->src + a, in));
      put32(o + 22 + cl, in);
      j->cblk[b] = o;
      j->clen[b] = total;
    }
  }
  return NULL;
}

static void run_jobs(job *jobs, int nt) {
  pthread_t th[256];
  for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
  for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
}

/* Records [lo, hi) of the n_records-record model as a run of BGZF blocks:
 * the BAM header first when with_header, the payload cut every block_payload
 * bytes with a short last block (the run ends at a record boundary, so the
 * runs of consecutive record ranges concatenate into one BAM), the EOF
 * block when p->eof_block.  Returns 0 on success. */
int gen_bam_segment(const gen_params *p, uint64_t lo, uint64_t hi, int with_header, uint8_t **out, uint64_t *out_len,
                    uint64_t *n_blocks, uint64_t *u_len) {
  model m;
  m.p = p;
  const uint64_t N = p->n_records;
  if (hi > N) hi = N;
  if (lo > hi) lo = hi;
  m.n_unplaced_start = p->mode != 1 ? N - N / 200 : N;
  m.n_mapped = m.n_unplaced_start;
  /* 30x local coverage of 150 bp reads: 5 bp per read */
  m.span = p->mode != 1 ? m.n_mapped * 5 : m.n_mapped * 1500;
  int nt = p->threads > 0 ? (p->threads > 256 ? 256 : p->threads) : 8;
  const uint64_t R = hi - lo;
  uint32_t *sizes = (uint32_t *)malloc((R + 1) * sizeof *sizes);
  uint64_t *offs = (uint64_t *)malloc((R + 1) * sizeof *offs);
  job jobs[256];
  for (int t = 0; t < nt; ++t) {
    memset(&jobs[t], 0, sizeof jobs[t]);
    jobs[t].m = &m;
    jobs[t].lo = lo + R * (uint64_t)t / (uint64_t)nt;
    jobs[t].hi = lo + R * (uint64_t)(t + 1) / (uint64_t)nt;
    jobs[t].base = lo;
    jobs[t].sizes = sizes;
    jobs[t].offs = offs;
    jobs[t].phase = 0;
  }
  run_jobs(jobs, nt);
  const size_t hl = with_header ? make_header(NULL) : 0;
  uint64_t u = hl;
  for (uint64_t i = 0; i < R; ++i) { offs[i] = u; u += sizes[i]; }
  uint8_t *ub = (uint8_t *)malloc(u + 16);
  if (!ub) return 1;
  if (with_header) make_header(ub);
  for (int t = 0; t < nt; ++t) { jobs[t].u = ub; jobs[t].phase = 1; }
  run_jobs(jobs, nt);
  const uint64_t nb = (u + (uint64_t)p->block_payload - 1) / (uint64_t)p->block_payload;
  uint8_t **cblk = (uint8_t **)calloc(nb + 1, sizeof *cblk);
  uint32_t *clen = (uint32_t *)calloc(nb + 1, sizeof *clen);
  for (int t = 0; t < nt; ++t) {
    jobs[t].phase = 2;
    jobs[t].src = ub;
    jobs[t].usz = u;
    jobs[t].blk_lo = nb * (uint64_t)t / (uint64_t)nt;
    jobs[t].blk_hi = nb * (uint64_t)(t + 1) / (uint64_t)nt;
    jobs[t].cblk = cblk;
    jobs[t].clen = clen;
  }
  run_jobs(jobs, nt);
  int err = 0;
  for (int t = 0; t < nt; ++t) err |= jobs[t].err;
  uint64_t tot = p->eof_block ? 28 : 0;
  for (uint64_t b = 0; b < nb; ++b) tot += clen[b];
  uint8_t *o = err ? NULL : (uint8_t *)malloc(tot ? tot : 1);
  uint64_t w = 0;
  for (uint64_t b = 0; b < nb; ++b) {
    if (o) memcpy(o + w, cblk[b], clen[b]);
    w += clen[b];
    free(cblk[b]);
  }
  if (o && p->eof_block) {
    static const uint8_t eofb[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    memcpy(o + w, eofb, 28);
  }
  free(cblk); free(clen); free(ub); free(sizes); free(offs);
  if (err) return 2;
  *out = o;
  *out_len = tot;
  if (n_blocks) *n_blocks = nb + (p->eof_block ? 1 : 0);
  if (u_len) *u_len = u;
  return 0;
}

/* Generate a whole BAM into a malloc'd buffer.  Returns 0 on success. */
int gen_bam(const gen_params *p, uint8_t **out, uint64_t *out_len, uint64_t *n_blocks, uint64_t *u_len) {
  return gen_bam_segment(p, 0, p->n_records, 1, out, out_len, n_blocks, u_len);
}

void gen_free(void *p) { free(p); }
