/*
 * orc_scan.c -- the restated CPU path over a whole file on many host threads.
 *
 * TEST INFRASTRUCTURE ONLY (see hbam_oracle.h): the nproc CPU baseline of
 * bench.py and the full-size checker of the 60 GB configurations (C3 decode
 * digests, C5 .splitting-bai bytes), where the single-threaded oracle would
 * need the whole inflated stream (~200 GB) in memory.
 *
 * It computes exactly what orc_decode_span (BAMRecordReader over [first
 * record, EOF)) and orc_splitting_index (SplittingBAMIndexer.index,
 * SplittingBAMIndexer.java:248-290) compute, streaming the file block by
 * block.  The record chain is sequential, so the file is cut into contiguous
 * block ranges, one per task: a task guesses where the chain enters its range
 * (the first position whose record and the next few records look valid, as
 * BAMSplitGuesser does), walks the chain through its range with zlib inflating
 * blocks on demand, and reports its exit.  A serial pass then checks every
 * guessed entry against the previous range's exit and re-walks the ranges
 * whose guess was off the chain, so the result never depends on the guess.
 * Empty mid-file blocks (htsjdk EOF) and malformed records end the chain as in
 * the single-threaded oracle; the scanner is meant for well-formed inputs and
 * reports ORC_E_FORMAT/TRUNC/ARG/IO at the first bad record otherwise.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "hbam_oracle.h"

static inline uint32_t s_rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline int32_t s_rdi32(const uint8_t *p) { return (int32_t)s_rd32(p); }

/* the order-sensitive digest of orc_scan_result (bench.py's 60 GB parity) */
static inline uint64_t s_dmix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
static uint64_t s_pow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  for (; e; e >>= 1, b *= b)
    if (e & 1) r *= b;
  return r;
}

typedef struct {
  uint64_t coff, ustart;
  uint32_t csize, isize;
} sblk;

typedef struct {
  const uint8_t *file;
  const sblk *b;
  uint64_t nb;
  /* inflated window: blocks [k0, k1) at buf[0 ..) */
  uint8_t *buf;
  uint64_t cap, k0, k1, u0, u1; /* u0 = ustart of k0, u1 = end of k1-1 */
} sreader;

static int sr_inflate_block(const uint8_t *f, const sblk *b, uint8_t *dst) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (inflateInit2(&z, -15) != Z_OK) return ORC_E_NOMEM;
  z.next_in = (Bytef *)(f + b->coff + 18);
  z.avail_in = b->csize - 26;
  z.next_out = dst;
  z.avail_out = b->isize;
  int rc = Z_OK;
  while (z.avail_out > 0) {
    rc = inflate(&z, Z_NO_FLUSH);
    if (rc != Z_OK || z.avail_in == 0) break;
  }
  const uint64_t got = b->isize - z.avail_out;
  inflateEnd(&z);
  if (rc != Z_OK && rc != Z_STREAM_END && rc != Z_BUF_ERROR) return ORC_E_IO;
  return got == b->isize ? ORC_OK : ORC_E_FORMAT;
}

/* make [pos, end) resident (end clipped to the stream); drops blocks before pos */
static int sr_need(sreader *r, uint64_t pos, uint64_t end, int *status) {
  if (r->k1 > r->k0 && pos >= r->u0) {
    /* drop whole blocks before pos */
    uint64_t k = r->k0;
    while (k < r->k1 && r->b[k].ustart + r->b[k].isize <= pos && r->b[k].ustart + r->b[k].isize < r->u1) k++;
    if (k > r->k0) {
      const uint64_t cut = r->b[k].ustart - r->u0;
      memmove(r->buf, r->buf + cut, r->u1 - r->b[k].ustart);
      r->u0 = r->b[k].ustart;
      r->k0 = k;
    }
  } else {
    /* restart at the block holding pos */
    uint64_t lo = 0, hi = r->nb;
    while (lo < hi) {
      uint64_t mid = (lo + hi) / 2;
      if (r->b[mid].ustart + r->b[mid].isize <= pos) lo = mid + 1; else hi = mid;
    }
    r->k0 = r->k1 = lo;
    r->u0 = r->u1 = lo < r->nb ? r->b[lo].ustart : pos;
  }
  while (r->u1 < end && r->k1 < r->nb) {
    const sblk *b = &r->b[r->k1];
    if (r->u1 - r->u0 + b->isize + 64 > r->cap) {
      uint64_t c = r->cap ? r->cap : (1 << 20);
      while (c < r->u1 - r->u0 + b->isize + 64) c *= 2;
      uint8_t *q = (uint8_t *)realloc(r->buf, c);
      if (!q) { *status = ORC_E_NOMEM; return 0; }
      r->buf = q;
      r->cap = c;
    }
    int rc = sr_inflate_block(r->file, b, r->buf + (r->u1 - r->u0));
    if (rc != ORC_OK) { *status = rc; return 0; }
    r->u1 += b->isize;
    r->k1++;
  }
  return r->u1 >= end;
}

static const uint8_t *sr_at(const sreader *r, uint64_t pos) { return r->buf + (pos - r->u0); }

typedef struct {
  /* shared */
  const uint8_t *file;
  const sblk *b;
  uint64_t nb, total_u;
  int32_t n_ref;
  const int32_t *ref_len;
  const uint64_t *dead;  /* sorted dead positions (empty block k >= 1) */
  uint64_t ndead;
  int mode, stringency;
  /* range */
  uint64_t lo_pos, hi_pos;  /* records starting in [lo_pos, hi_pos) belong here */
  uint64_t entry;           /* chain position entering the range (guess or true) */
  int guessed;              /* entry is a guess */
  int seek_start;           /* the range starts at the reader's seek (the first record) */
  /* results */
  uint64_t exit;            /* first chain position >= hi_pos (or where it stopped) */
  int stopped;              /* the chain ended inside the range (EOF / error) */
  int status;
  uint64_t n, key_xor, voff_sum;
  uint64_t kdig, vdig;      /* order-sensitive digests of this range (Horner) */
  uint64_t fdig[ORC_N_FIELDS]; /* the same of each fixed field (orc_scan_result.field_digest order) */
  uint32_t rcrc;            /* zlib crc32 of the records' rests, back to back */
  uint64_t rlen;            /* their bytes */
  uint64_t *voffs, vcap;    /* index mode (and keep): every record voff */
  int64_t *keys;            /* decode mode with keep: every record key (capacity vcap) */
  int keep;                 /* decode mode: keep every voff and key */
} stask;

static int is_dead_pos(const stask *t, uint64_t q) {
  uint64_t lo = 0, hi = t->ndead;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (t->dead[mid] < q) lo = mid + 1; else hi = mid;
  }
  return lo < t->ndead && t->dead[lo] == q;
}

/* normalized voff of stream position q ([htsjdk] getFilePointer) */
static uint64_t s_voff(const stask *t, uint64_t q) {
  uint64_t lo = 0, hi = t->nb;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (t->b[mid].ustart >= q) hi = mid; else lo = mid + 1;
  }
  if (lo < t->nb && t->b[lo].ustart == q) return t->b[lo].coff << 16;
  const sblk *b = &t->b[lo - 1];
  if (q - b->ustart < b->isize) return (b->coff << 16) | (q - b->ustart);
  return (b->coff + b->csize) << 16;
}

/* a record start that looks valid, and the next 4 after it */
static int s_plausible_at(sreader *r, const stask *t, uint64_t q, int *st) {
  uint64_t p = q;
  for (int k = 0; k < 5; k++) {
    if (p == t->total_u) return k > 0;
    if (!sr_need(r, p, p + 36, st)) return k > 0 && *st == ORC_OK;
    const uint8_t *x = sr_at(r, p);
    const int32_t bs = s_rdi32(x), ref = s_rdi32(x + 4), pos = s_rdi32(x + 8), lseq = s_rdi32(x + 20);
    const int32_t nref = s_rdi32(x + 24), npos = s_rdi32(x + 28);
    const int64_t lrn = x[12], ncig = x[16] | (x[17] << 8);
    if (ref < -1 || ref >= t->n_ref || nref < -1 || nref >= t->n_ref || pos < -1 || npos < -1) return 0;
    if (lrn < 1 || lseq < 0 || bs < 32 + lrn + 4 * ncig + lseq + (lseq + 1) / 2) return 0;
    if (p + 4 + (uint64_t)bs > t->total_u) return 0;
    if (!sr_need(r, p, p + 36 + lrn, st)) return 0;
    if (sr_at(r, p)[36 + lrn - 1] != 0) return 0;
    p += 4 + (uint64_t)bs;
  }
  return 1;
}

/* walk the chain from t->entry over the range; returns 0 or a fatal status */
static void s_walk(stask *t, sreader *r) {
  uint64_t q = t->entry;
  t->n = t->key_xor = t->voff_sum = 0;
  t->kdig = t->vdig = 0;
  memset(t->fdig, 0, sizeof t->fdig);
  t->rcrc = (uint32_t)crc32(0L, Z_NULL, 0);
  t->rlen = 0;
  t->stopped = 0;
  t->status = ORC_OK;
  int first = 1;  /* reader: the split start follows a seek (no dead check) */
  while (q < t->hi_pos) {
    if (q >= t->total_u) { t->stopped = 1; break; }
    if (!(t->mode == 0 && first && t->seek_start) && is_dead_pos(t, q)) { t->stopped = 1; break; }
    first = 0;
    const uint64_t avail = t->total_u - q;
    int st = ORC_OK;
    if (avail < 4) {
      if (t->mode == 1) t->status = ORC_E_IO; /* "less than 4 bytes long" */
      t->stopped = 1;
      break;
    }
    if (!sr_need(r, q, q + 4, &st)) { t->status = st ? st : ORC_E_TRUNC; t->stopped = 1; break; }
    const int32_t bs = s_rdi32(sr_at(r, q));
    const uint64_t v = s_voff(t, q);
    if (t->mode == 0) {
      if (bs < 32) { t->status = ORC_E_FORMAT; t->stopped = 1; break; }
      if (avail - 4 < (uint64_t)bs) { t->status = ORC_E_TRUNC; t->stopped = 1; break; }
      /* an empty block where one of BAMRecordCodec.decode's reads starts */
      static const uint8_t starts[] = {4, 8, 12, 13, 14, 16, 18, 20, 24, 28, 32, 36};
      for (unsigned k = 0; k < sizeof starts && !t->stopped; k++)
        if ((starts[k] < 36 || bs > 32) && is_dead_pos(t, q + starts[k])) { t->status = ORC_E_TRUNC; t->stopped = 1; }
      if (t->stopped) break;
      if (!sr_need(r, q, q + 4 + (uint64_t)bs, &st)) { t->status = st ? st : ORC_E_TRUNC; t->stopped = 1; break; }
      const uint8_t *x = sr_at(r, q);
      const int32_t ref = s_rdi32(x + 4), nref = s_rdi32(x + 24);
      if (ref < -1 || ref >= t->n_ref || nref < -1 || nref >= t->n_ref) { t->status = ORC_E_ARG; t->stopped = 1; break; }
      if (t->stringency != ORC_SILENT &&
          orc_record_invalid(x, bs, t->n_ref, t->ref_len, t->stringency == ORC_STRICT)) {
        t->status = ORC_E_FORMAT;
        t->stopped = 1;
        break;
      }
      const uint16_t flag = (uint16_t)(x[18] | (x[19] << 8));
      const uint64_t key = (uint64_t)orc_get_key(ref, s_rdi32(x + 8), flag, x + 36, (uint32_t)(bs - 32));
      t->key_xor ^= key;
      t->voff_sum += v;
      t->kdig = t->kdig * ORC_DIGEST_P + s_dmix(key);
      t->vdig = t->vdig * ORC_DIGEST_P + s_dmix(v);
      /* the fixed fields (signed ones sign-extended to 64 bits) and the rest
       * (LazyBAMRecordFactory.createBAMRecord's arguments) */
      const uint64_t fv[ORC_N_FIELDS] = {
          (uint64_t)(int64_t)ref, (uint64_t)(int64_t)s_rdi32(x + 8), x[12], x[13], (uint64_t)(x[14] | (x[15] << 8)),
          (uint64_t)(x[16] | (x[17] << 8)), flag, (uint64_t)(int64_t)s_rdi32(x + 20), (uint64_t)(int64_t)nref,
          (uint64_t)(int64_t)s_rdi32(x + 28), (uint64_t)(int64_t)s_rdi32(x + 32)};
      for (int f = 0; f < ORC_N_FIELDS; f++) t->fdig[f] = t->fdig[f] * ORC_DIGEST_P + s_dmix(fv[f]);
      t->rcrc = (uint32_t)crc32(t->rcrc, x + 36, (uInt)(bs - 32));
      t->rlen += (uint64_t)(bs - 32);
      if (t->keep) {
        if (t->n == t->vcap) {
          t->vcap = t->vcap ? 2 * t->vcap : 1 << 16;
          uint64_t *nv = (uint64_t *)realloc(t->voffs, t->vcap * 8);
          int64_t *nk = (int64_t *)realloc(t->keys, t->vcap * 8);
          if (nv) t->voffs = nv;
          if (nk) t->keys = nk;
          if (!nv || !nk) { t->status = ORC_E_NOMEM; t->stopped = 1; break; }
        }
        t->voffs[t->n] = v;
        t->keys[t->n] = (int64_t)key;
      }
      t->n++;
      q += 4 + (uint64_t)bs;
    } else {
      if (t->n == t->vcap) {
        t->vcap = t->vcap ? 2 * t->vcap : 1 << 16;
        uint64_t *nv = (uint64_t *)realloc(t->voffs, t->vcap * 8);
        if (!nv) { t->status = ORC_E_NOMEM; t->stopped = 1; break; }
        t->voffs = nv;
      }
      t->voffs[t->n++] = v;
      t->voff_sum += v;
      t->vdig = t->vdig * ORC_DIGEST_P + s_dmix(v);
      q += 4;
      if (bs > 0) {
        if ((uint64_t)bs > avail - 4 || is_dead_pos(t, q)) { t->status = ORC_E_IO; t->stopped = 1; break; } /* Skip failed */
        q += (uint64_t)bs;
      }
    }
  }
  t->exit = q;
}

typedef struct {
  stask *tasks;
  int ntask, next;
  pthread_mutex_t mu;
} spool;

static void *s_worker(void *arg) {
  spool *P = (spool *)arg;
  sreader r;
  memset(&r, 0, sizeof r);
  for (;;) {
    pthread_mutex_lock(&P->mu);
    const int i = P->next++;
    pthread_mutex_unlock(&P->mu);
    if (i >= P->ntask) break;
    stask *t = &P->tasks[i];
    r.file = t->file;
    r.b = t->b;
    r.nb = t->nb;
    r.k0 = r.k1 = 0;
    r.u0 = r.u1 = 0;
    if (t->guessed) { /* first position of the range that starts a plausible chain */
      int st = ORC_OK;
      uint64_t q = t->lo_pos, found = UINT64_MAX;
      const uint64_t lim = t->hi_pos < t->total_u ? t->hi_pos : t->total_u;
      for (; q < lim; q++)
        if (s_plausible_at(&r, t, q, &st)) { found = q; break; }
      t->entry = found == UINT64_MAX ? t->hi_pos : found;
    }
    s_walk(t, &r);
  }
  free(r.buf);
  return NULL;
}

static int scan_impl(const uint8_t *file, uint64_t len, int threads, int mode, int stringency, int32_t g,
                     uint64_t max_blocks, uint8_t **sbi, uint64_t *sbi_len, orc_scan_result *res, int64_t *keys_out,
                     uint64_t *voffs_out, uint64_t out_cap) {
  memset(res, 0, sizeof *res);
  if (sbi) { *sbi = NULL; *sbi_len = 0; }
  if (mode == 1 && g <= 0) return ORC_E_ARG;
  /* block table (BSIZE walk; framing as the single-threaded oracle) */
  uint64_t cap = 1 << 16, nb = 0, p = 0, u = 0;
  sblk *b = (sblk *)malloc(cap * sizeof *b);
  while (p < len && (!max_blocks || nb < max_blocks)) {
    if (len - p < 18) { free(b); return ORC_E_IO; }
    const uint8_t *h = file + p;
    const uint32_t total = (uint32_t)(h[16] | (h[17] << 8)) + 1;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4 || (h[10] | (h[11] << 8)) != 6 || total < 26) {
      free(b);
      return ORC_E_FORMAT;
    }
    if (p + total > len) { free(b); return ORC_E_TRUNC; }
    if (nb == cap) b = (sblk *)realloc(b, (cap *= 2) * sizeof *b);
    b[nb].coff = p;
    b[nb].csize = total;
    b[nb].isize = s_rd32(h + total - 4);
    b[nb].ustart = u;
    u += b[nb].isize;
    p += total;
    nb++;
  }
  const uint64_t flen = max_blocks && nb == max_blocks ? p : len;
  /* header ([htsjdk] BAMFileReader.readHeader) from the first blocks */
  sreader hr;
  memset(&hr, 0, sizeof hr);
  hr.file = file;
  hr.b = b;
  hr.nb = nb;
  int st = ORC_OK;
  uint64_t hp = 8;
  int32_t n_ref = 0;
  int32_t *ref_len = NULL;
  if (!sr_need(&hr, 0, 8, &st) || memcmp(hr.buf, "BAM\1", 4) != 0) { free(b); free(hr.buf); return ORC_E_IO; }
  hp += (uint64_t)s_rdi32(hr.buf + 4);
  if (!sr_need(&hr, 0, hp + 4, &st)) { free(b); free(hr.buf); return ORC_E_TRUNC; }
  n_ref = s_rdi32(hr.buf + hp);
  hp += 4;
  ref_len = (int32_t *)calloc(n_ref > 0 ? (size_t)n_ref : 1, 4);
  for (int32_t i = 0; i < n_ref; i++) {
    if (!sr_need(&hr, 0, hp + 4, &st)) { free(b); free(hr.buf); free(ref_len); return ORC_E_TRUNC; }
    const uint64_t ln = (uint64_t)s_rdi32(hr.buf + hp);
    if (!sr_need(&hr, 0, hp + 8 + ln, &st)) { free(b); free(hr.buf); free(ref_len); return ORC_E_TRUNC; }
    ref_len[i] = s_rdi32(hr.buf + hp + 4 + ln);
    hp += 8 + ln;
  }
  free(hr.buf);
  const uint64_t header_end = hp;
  /* dead positions: an empty block k >= 1 */
  uint64_t *dead = (uint64_t *)malloc((nb + 1) * 8), ndead = 0;
  for (uint64_t k = 1; k < nb; k++)
    if (b[k].isize == 0 && (ndead == 0 || dead[ndead - 1] != b[k].ustart)) dead[ndead++] = b[k].ustart;
  /* ranges of about equal compressed size: 4 per thread */
  if (threads < 1) threads = 1;
  int ntask = threads == 1 ? 1 : threads * 4;
  if ((uint64_t)ntask > nb) ntask = nb ? (int)nb : 1;
  stask *T = (stask *)calloc((size_t)ntask, sizeof *T);
  uint64_t kb = 0;
  for (int i = 0; i < ntask; i++) {
    uint64_t ke = i + 1 == ntask ? nb : kb;
    const uint64_t target = flen * (uint64_t)(i + 1) / (uint64_t)ntask;
    while (ke < nb && b[ke].coff < target) ke++;
    stask *t = &T[i];
    t->file = file;
    t->b = b;
    t->nb = nb;
    t->total_u = u;
    t->n_ref = n_ref;
    t->ref_len = ref_len;
    t->dead = dead;
    t->ndead = ndead;
    t->mode = mode;
    t->stringency = stringency;
    t->lo_pos = kb < nb ? b[kb].ustart : u;
    t->hi_pos = ke < nb ? b[ke].ustart : u;
    if (t->lo_pos < header_end) t->lo_pos = header_end;
    if (t->hi_pos < t->lo_pos) t->hi_pos = t->lo_pos;
    t->entry = t->lo_pos;
    t->guessed = i > 0;
    t->seek_start = i == 0;
    t->keep = mode == 0 && keys_out != NULL;
    kb = ke;
  }
  spool P = {T, ntask, 0, PTHREAD_MUTEX_INITIALIZER};
  pthread_t *th = (pthread_t *)malloc((size_t)threads * sizeof *th);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, s_worker, &P);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  /* serial link: each range must start where the previous one's chain left */
  int rc = ORC_OK, ended = 0;
  sreader rr;
  memset(&rr, 0, sizeof rr);
  rr.file = file;
  rr.b = b;
  rr.nb = nb;
  uint64_t ordinal = 0;
  uint64_t *ent = NULL, nent = 0, entcap = 0;
  uint64_t first_voff = 0;
  {
    stask tmp = T[0];
    first_voff = s_voff(&tmp, header_end);
  }
  for (int i = 0; i < ntask && !ended; i++) {
    stask *t = &T[i];
    if (i > 0) {
      const stask *pv = &T[i - 1];
      if (t->entry != pv->exit) { /* the guess was off the chain: re-walk from the true entry */
        t->entry = pv->exit;
        t->guessed = 0;
        if (t->entry < t->hi_pos) {
          res->rewalks++;
          s_walk(t, &rr);
        } else { /* the previous chain jumped over this whole range */
          t->n = 0;
          t->key_xor = t->voff_sum = 0;
          t->kdig = t->vdig = 0;
          memset(t->fdig, 0, sizeof t->fdig);
          t->rcrc = (uint32_t)crc32(0L, Z_NULL, 0);
          t->rlen = 0;
          t->exit = t->entry;
          t->stopped = 0;
          t->status = ORC_OK;
        }
      }
    }
    if (t->keep) {
      if (res->records + t->n > out_cap) {
        rc = ORC_E_NOMEM;
        break;
      }
      memcpy(voffs_out + res->records, t->voffs, t->n * 8);
      memcpy(keys_out + res->records, t->keys, t->n * 8);
    }
    res->records += t->n;
    res->key_xor ^= t->key_xor;
    res->voff_sum += t->voff_sum;
    const uint64_t w = s_pow(ORC_DIGEST_P, t->n);
    res->key_digest = res->key_digest * w + t->kdig;
    res->voff_digest = res->voff_digest * w + t->vdig;
    for (int f = 0; f < ORC_N_FIELDS; f++) res->field_digest[f] = res->field_digest[f] * w + t->fdig[f];
    res->rest_crc = res->rest_bytes ? (uint32_t)crc32_combine(res->rest_crc, t->rcrc, (z_off_t)t->rlen) : t->rcrc;
    res->rest_bytes += t->rlen;
    if (mode == 1 && sbi) {
      for (uint64_t j = 0; j < t->n; j++) {
        if ((ordinal + j + 1) % (uint64_t)g == 0) {
          if (nent == entcap) ent = (uint64_t *)realloc(ent, (entcap = entcap ? 2 * entcap : 1024) * 8);
          ent[nent++] = t->voffs[j];
        }
      }
    }
    ordinal += t->n;
    if (t->stopped) {
      ended = 1;
      rc = t->status;
    }
  }
  free(rr.buf);
  res->blocks = nb;
  res->u_bytes = u;
  res->status = rc;
  if (rc == ORC_OK && mode == 1 && sbi) {
    const uint64_t n = nent + 2;
    uint8_t *o = (uint8_t *)malloc(n * 8);
    uint64_t vals[2] = {first_voff, flen << 16};
    for (uint64_t k = 0; k < n; k++) {
      const uint64_t v = k == 0 ? vals[0] : k == n - 1 ? vals[1] : ent[k - 1];
      for (int q = 0; q < 8; q++) o[8 * k + q] = (uint8_t)(v >> (56 - 8 * q));
    }
    *sbi = o;
    *sbi_len = n * 8;
  }
  free(ent);
  for (int i = 0; i < ntask; i++) {
    free(T[i].voffs);
    free(T[i].keys);
  }
  free(T);
  free(dead);
  free(ref_len);
  free(b);
  return rc;
}

int orc_scan(const uint8_t *file, uint64_t len, int threads, int mode, int stringency, int32_t g,
             uint64_t max_blocks, uint8_t **sbi, uint64_t *sbi_len, orc_scan_result *res) {
  return scan_impl(file, len, threads, mode, stringency, g, max_blocks, sbi, sbi_len, res, NULL, NULL, 0);
}

int orc_scan_records(const uint8_t *file, uint64_t len, int threads, int stringency, uint64_t cap, int64_t *keys,
                     uint64_t *voffs, orc_scan_result *res) {
  return scan_impl(file, len, threads, 0, stringency, 0, 0, NULL, NULL, res, keys, voffs, cap);
}
