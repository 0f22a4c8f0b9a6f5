// hbam_abi.cpp -- extern "C" boundary (include/hbam.h) over the C++ mirror.
#include "../../include/hbam.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "hbam_deflate_api.h"
#include "hbam_mem.h"
#include "hbam_host.h"
#include "hbam_launch.h"

using hadoop_bam::BAMInputFormat;
using hadoop_bam::BamFile;
using hadoop_bam::BAMRecordReader;
using hadoop_bam::Carry;
using hadoop_bam::FileSplit;
using hadoop_bam::FileVirtualSplit;
using hadoop_bam::HostBatch;
using hadoop_bam::OpenOptions;
using hadoop_bam::SpanCursor;
using hadoop_bam::SplittingBAMIndexer;
using hadoop_bam::Step;

struct hbam_ctx {
  std::unique_ptr<BamFile> f;
  std::unique_ptr<hbam::Pipeline> codec;  // hbam_open_codec: a pipeline with no file
  std::string err;
  SpanCursor cursor;    // (destroyed before f: it drains its copies on f's pipeline stream)
  HostBatch wbatch;     // the columns of the last hbam_decode_writables
  hadoop_bam::BatchView batch;  // the last batch handed out (cursor slots or wbatch)
  hbam::SpanDev wspan;  // device result of the last hbam_decode_writables
  bool last_is_writables = false;
};

struct hbam_gpu {
  std::unique_ptr<BamFile> f;
  int device = 0;
  uint64_t window = hadoop_bam::kDefaultWindowBytes;
  std::string err;
  hbam::SpanDev span;  // last window of the last run
  hbam::DevBuf<uint8_t> enc;  // hbam_gpu_encode_writables output
  uint64_t enc_bytes = 0;
  std::unique_ptr<hbam::BgzfCompressor> bgzf;  // hbam_gpu_bgzf_compress
};

namespace {
// the last error of a call with no ctx (open, compress, codec): per thread,
// as JNI callers from many executor threads read it right after their call
thread_local std::string g_open_err;

OpenOptions options_of(const hbam_opts* opts, bool header) {
  hbam_opts o{};
  if (opts) o = *opts;
  OpenOptions r;
  r.device = o.device;
  r.check_crc = o.check_crc != 0;
  r.stringency = o.stringency;
  r.window_bytes = o.window_bytes;
  r.parallel_reads = o.parallel_reads != 0;
  r.batch_records = o.batch_records;
  r.parse_header = header;
  return r;
}

int finish_open(int rc, std::unique_ptr<BamFile>&& f, const std::string& err, hbam_ctx** out,
                const hbam_opts* opts = nullptr) {
  auto* c = new hbam_ctx();
  *out = c;  // on failure the caller may read hbam_last_error, then must hbam_close
  if (rc != HBAM_OK) {
    g_open_err = err;
    c->err = err;
    return rc;
  }
  c->f = std::move(f);
  // the caller's batch size is known: its page-locked batch slots are pinned
  // on a helper thread while it goes on (the first hbam_decode_span joins it)
  if (opts && opts->batch_records) c->cursor.start_prealloc(opts->batch_records, opts->device);
  return HBAM_OK;
}

bool valid_stringency(const hbam_opts* o) { return !o || (o->stringency >= 0 && o->stringency <= 2); }

void fill_batch(const hadoop_bam::BatchView& h, hbam_batch* out) {
  out->n = h.n;
  out->ref_id = h.ref_id;
  out->pos = h.pos;
  out->l_seq = h.l_seq;
  out->next_ref_id = h.next_ref_id;
  out->next_pos = h.next_pos;
  out->tlen = h.tlen;
  out->l_read_name = h.l_read_name;
  out->mapq = h.mapq;
  out->bin = h.bin;
  out->n_cigar = h.n_cigar;
  out->flag = h.flag;
  out->key = h.key;
  out->voff = h.voff;
  out->rest_off = h.rest_off;
  out->rest_len = h.rest_len;
  out->data = h.data;
  out->data_len = h.data_len;
}

// The decode of FileVirtualSplit [vstart, vend) window by window with the
// records left in HBM; stats accumulate over windows.  *last = the last
// window's span (C2-sized files: the whole split).
int decode_device(BamFile& f, uint64_t vstart, uint64_t vend, int32_t flags, hbam_gpu_stats* st,
                  hbam::SpanDev* last, std::string* err) {
  memset(st, 0, sizeof *st);
  hbam::Pipeline& p = f.pipe();
  p.timing = (flags & 1) != 0;
  const bool decode = (flags & 2) == 0, digest = (flags & 4) != 0;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, p.stream());
  const uint64_t lf0 = p.link_fallbacks(), il0 = p.inflate_launches(), lr0 = p.link_rewalks();
  const uint64_t rf0 = p.record_fallbacks();
  f.invalidate_window();  // a timed pass locates and inflates afresh
  Carry c{vstart >> 16, vstart & 0xffff};
  bool cont = false;
  int rc = HBAM_OK;
  bool first = true;
  // Windows read from the host ramp up (SpanCursor::ramp_window: 32 MiB,
  // doubling to the full window), so that decoding starts after the first
  // small copy instead of a whole 4 GiB window's (C3 from the mapped file);
  // a span already in HBM decodes in full windows.
  const uint64_t span_end = std::min<uint64_t>(f.file_size(), vend == ~0ull ? ~0ull : (vend >> 16) + 0x20000);
  const bool ramp = !f.window_explicit() && !f.resident(vstart >> 16, span_end);
  uint64_t nwin = 0;
  for (;;) {
    Step step;
    rc = ramp ? f.decode_step(c, vend, hbam::kReader, decode, cont, &step,
                              hadoop_bam::SpanCursor::ramp_window(f.window_bytes(), nwin),
                              hadoop_bam::SpanCursor::ramp_window(f.window_bytes(), nwin + 1))
              : f.decode_step(c, vend, hbam::kReader, decode, cont, &step);
    ++nwin;
    if (rc != HBAM_OK) {
      *err = f.error();
      break;
    }
    const hbam::SpanDev& s = step.span;
    st->windows += 1;
    st->records += s.n;
    st->n_blocks += p.blocks().size();
    // bytes of this window up to the block the next window starts at (it
    // starts at the record this one could not finish): each counted once
    const bool last_window = step.ended || step.status != HBAM_OK;
    const int64_t next_u = last_window ? -1 : p.pos_of_voff(step.next.coff << 16);
    if (next_u < 0) {
      st->compressed_bytes += p.window_end() - c.coff;
      st->inflated_bytes += p.total_u();
    } else {
      st->compressed_bytes += step.next.coff - c.coff;
      st->inflated_bytes += (uint64_t)next_u;
    }
    if (p.timing) {
      st->ms_locate += p.times.locate;
      st->ms_inflate += p.times.inflate;
      st->ms_huff += p.times.huff;
      st->ms_lz77 += p.times.lz77;
      st->ms_tables += p.times.tables;
      st->ms_chain += p.times.chain;
      st->ms_decode += p.times.decode;
    }
    if (s.n) {
      if (first) st->first_voff = s.first_voff;
      st->last_voff = s.last_voff;
      first = false;
      if (digest) {
        uint64_t dg[4];
        hbam::SpanDev d = s;
        if (!decode) d.col.key = nullptr;
        rc = p.span_digest(d, dg);
        if (rc != HBAM_OK) {
          *err = p.error();
          break;
        }
        st->key_xor ^= dg[0];
        st->voff_sum += dg[1];
        uint64_t w = 1, b = HBAM_DIGEST_P;  // P^n of this window's records
        for (uint64_t e = s.n; e; e >>= 1, b *= b)
          if (e & 1) w *= b;
        st->key_digest = st->key_digest * w + dg[2];
        st->voff_digest = st->voff_digest * w + dg[3];
      }
    }
    if (last) *last = s;
    if (step.status != HBAM_OK) {
      st->status = step.status;
      *err = step.error;
      break;
    }
    if (step.ended) break;
    c = step.next;
    cont = true;
  }
  (void)hipEventRecord(e1, p.stream());
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&st->ms_total, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  st->link_fallbacks = (int32_t)(p.link_fallbacks() - lf0);
  st->inflate_launches = (int32_t)(p.inflate_launches() - il0);
  st->link_rewalks = (int32_t)(p.link_rewalks() - lr0);
  st->record_fallbacks = (int32_t)(p.record_fallbacks() - rf0);
  if (rc != HBAM_OK) st->status = rc;
  return rc != HBAM_OK ? rc : st->status;
}
// page-locked blocks handed out by hbam_host_alloc and their sizes (pinned_free needs them)
std::mutex& host_alloc_mu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
std::map<void*, size_t>& host_allocs() {
  static std::map<void*, size_t>* m = new std::map<void*, size_t>();
  return *m;
}

}  // namespace

extern "C" {

int32_t hbam_abi_version(void) { return HBAM_ABI_VERSION; }

int hbam_open_mem(const void* data, uint64_t len, const hbam_opts* opts, hbam_ctx** out) {
  if (!valid_stringency(opts)) return finish_open(HBAM_E_ARG, nullptr, "unknown validation stringency", out);
  std::unique_ptr<BamFile> f;
  std::string err;
  int rc = BamFile::open_memory(static_cast<const uint8_t*>(data), len, options_of(opts, true), &f, &err);
  return finish_open(rc, std::move(f), err, out, opts);
}

int hbam_open_bgzf(const void* data, uint64_t len, const hbam_opts* opts, hbam_ctx** out) {
  std::unique_ptr<BamFile> f;
  std::string err;
  int rc = BamFile::open_memory(static_cast<const uint8_t*>(data), len, options_of(opts, false), &f, &err);
  return finish_open(rc, std::move(f), err, out, opts);
}

int hbam_open(const char* path, const hbam_opts* opts, hbam_ctx** out) {
  if (!valid_stringency(opts)) return finish_open(HBAM_E_ARG, nullptr, "unknown validation stringency", out);
  std::unique_ptr<BamFile> f;
  std::string err;
  int rc = BamFile::open_path(path, options_of(opts, true), &f, &err);
  return finish_open(rc, std::move(f), err, out, opts);
}

int hbam_open_reader(uint64_t size, hbam_read_fn read, void* user, const hbam_opts* opts, hbam_ctx** out) {
  if (!valid_stringency(opts)) return finish_open(HBAM_E_ARG, nullptr, "unknown validation stringency", out);
  if (!read) return finish_open(HBAM_E_ARG, nullptr, "no reader", out);
  std::unique_ptr<BamFile> f;
  std::string err;
  int rc = BamFile::open_reader(size, read, user, options_of(opts, true), &f, &err);
  return finish_open(rc, std::move(f), err, out, opts);
}

void hbam_close(hbam_ctx* ctx) { delete ctx; }

const char* hbam_last_error(hbam_ctx* ctx) { return ctx ? ctx->err.c_str() : g_open_err.c_str(); }

void hbam_free(void* p) { free(p); }

uint64_t hbam_release_cached_memory(void) { return hbam::release_cached(); }

int hbam_bgzf_compress(const hbam_opts* opts, const void* data, uint64_t len, const uint32_t* block_lens,
                       uint64_t n_blocks, int32_t block_size, int32_t level, int32_t flags, uint8_t** out,
                       uint64_t* out_len) {
  *out = nullptr;
  *out_len = 0;
  hbam_opts o{};
  if (opts) o = *opts;
  std::vector<uint64_t> ustart;
  std::vector<uint32_t> lens;
  uint64_t pos = 0;
  if (block_lens) {
    for (uint64_t i = 0; i < n_blocks; ++i) {
      ustart.push_back(pos);
      lens.push_back(block_lens[i]);
      pos += block_lens[i];
    }
    if (pos != len) {
      g_open_err = "block_lens do not sum to len";
      return HBAM_E_ARG;
    }
  } else {
    if (block_size <= 0 || block_size > 65536) {
      g_open_err = "block_size must be 1..65536";
      return HBAM_E_ARG;
    }
    for (; pos < len; pos += (uint64_t)block_size) {
      ustart.push_back(pos);
      lens.push_back((uint32_t)std::min<uint64_t>((uint64_t)block_size, len - pos));
    }
  }
  if (o.device < 0 || o.device >= hbam_device_count()) {
    g_open_err = "no HIP device " + std::to_string(o.device);
    return HBAM_E_DEVICE;
  }
  if (hipSetDevice(o.device) != hipSuccess) return HBAM_E_DEVICE;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return HBAM_E_DEVICE;
  uint8_t* d_in = nullptr;
  int rc = HBAM_OK;
  if (hipMalloc(reinterpret_cast<void**>(&d_in), len + 64) != hipSuccess ||  // 64 B pad: deflate's 8-byte compares
      (len && hipMemcpyAsync(d_in, data, len, hipMemcpyHostToDevice, s) != hipSuccess)) {
    g_open_err = "device buffer for the payload";
    rc = HBAM_E_DEVICE;
  }
  {
    hbam::BgzfCompressor c(o.device);
    if (rc == HBAM_OK) {
      rc = c.compress(d_in, ustart, lens, level, (flags & HBAM_BGZF_EOF) != 0, s, nullptr);
      if (rc != HBAM_OK) g_open_err = c.error();
    }
    if (rc == HBAM_OK) {
      uint8_t* h = static_cast<uint8_t*>(malloc(c.out_len() ? c.out_len() : 1));
      if (!h) {
        rc = HBAM_E_NOMEM;
      } else if (c.out_len() && hipMemcpy(h, c.d_out(), c.out_len(), hipMemcpyDeviceToHost) != hipSuccess) {
        free(h);
        rc = HBAM_E_DEVICE;
      } else {
        *out = h;
        *out_len = c.out_len();
      }
    }
  }
  if (d_in) (void)hipFree(d_in);
  (void)hipStreamDestroy(s);
  return rc;
}

int hbam_header(hbam_ctx* ctx, hbam_header_info* out) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  BamFile& f = *ctx->f;
  out->n_ref = f.n_ref();
  out->l_text = f.l_text();
  out->first_record_voff = f.first_record_voff();
  out->file_size = f.file_size();
  out->text = f.text().c_str();
  return HBAM_OK;
}

int hbam_ref(hbam_ctx* ctx, int32_t i, const char** name, int32_t* length) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  if (i < 0 || i >= ctx->f->n_ref()) {
    ctx->err = "reference index out of range";
    return HBAM_E_ARG;
  }
  *name = ctx->f->ref_names()[(size_t)i].c_str();
  *length = ctx->f->ref_lens()[(size_t)i];
  return HBAM_OK;
}

int hbam_file_stats(hbam_ctx* ctx, uint64_t* n_blocks, uint64_t* uncompressed_size) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();  // all_blocks() moves the window
  const std::vector<hbam::BlockInfo>* B = nullptr;
  int rc = ctx->f->all_blocks(&B);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  *n_blocks = B->size();
  *uncompressed_size = B->empty() ? 0 : B->back().ustart + B->back().isize;
  return HBAM_OK;
}

int hbam_bytes_read(hbam_ctx* ctx, uint64_t* bytes) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  *bytes = ctx->f->bytes_read();
  return HBAM_OK;
}

int hbam_prefetch(hbam_ctx* ctx, uint64_t lo, uint64_t hi) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  if (hi < lo) {
    ctx->err = "prefetch range end before its start";
    return HBAM_E_ARG;
  }
  ctx->cursor.reset();
  int rc = ctx->f->prefetch(lo, hi);
  if (rc != HBAM_OK) ctx->err = ctx->f->error();
  return rc;
}

int hbam_decode_span(hbam_ctx* ctx, uint64_t vstart, uint64_t vend, uint64_t max_records, hbam_batch* out) {
  memset(out, 0, sizeof *out);
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->last_is_writables = false;
  uint64_t next = vend;
  int rc = ctx->cursor.next_batch(*ctx->f, vstart, vend, max_records, &ctx->batch, &next, &ctx->err);
  fill_batch(ctx->batch, out);
  out->next_voff = next;
  out->status = rc;
  if (rc == HBAM_E_DEVICE || rc == HBAM_E_STATE || rc == HBAM_E_NOMEM) out->n = 0;
  return rc;
}

int hbam_reader_position(hbam_ctx* ctx, uint64_t i, uint64_t* pos) {
  *pos = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  if (ctx->last_is_writables || !ctx->cursor.valid()) {
    ctx->err = "hbam_reader_position needs the last call on the ctx to be hbam_decode_span";
    return HBAM_E_STATE;
  }
  if (i == UINT64_MAX) return ctx->cursor.initial_position(pos, &ctx->err);  // before record 0 is handed out
  if (i >= ctx->batch.n) {
    ctx->err = "record index outside the last batch";
    return HBAM_E_ARG;
  }
  return ctx->cursor.reader_position(i, pos, &ctx->err);
}

int hbam_pipeline_counters(hbam_ctx* ctx, uint64_t out[5]) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  hbam::Pipeline& p = ctx->f->pipe();
  out[0] = p.link_fallbacks();
  out[1] = p.link_rewalks();
  out[2] = p.record_fallbacks();
  out[3] = p.inflate_launches();
  out[4] = p.records_after_stop();
  return HBAM_OK;
}

int hbam_inflate_token_count(hbam_ctx* ctx, uint64_t* tokens) {
  *tokens = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  return ctx->f->pipe().inflate_tokens(tokens) == 0 ? HBAM_OK : HBAM_E_DEVICE;
}

int hbam_decode_span_device(hbam_ctx* ctx, uint64_t vstart, uint64_t vend, int32_t flags, hbam_gpu_stats* st) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  return decode_device(*ctx->f, vstart, vend, flags, st, nullptr, &ctx->err);
}

int hbam_open_codec(const hbam_opts* opts, hbam_ctx** out) {
  *out = nullptr;
  hbam_opts o{};
  if (opts) o = *opts;
  if (o.device < 0 || o.device >= hbam_device_count()) {
    g_open_err = "no HIP device " + std::to_string(o.device);
    return HBAM_E_DEVICE;
  }
  auto* c = new hbam_ctx();
  c->codec.reset(new hbam::Pipeline(o.device));
  *out = c;
  if (!c->codec->error().empty()) {
    c->err = g_open_err = c->codec->error();
    return HBAM_E_DEVICE;
  }
  return HBAM_OK;
}

int hbam_encode_writables(hbam_ctx* ctx, uint8_t* out, uint64_t cap, uint64_t* offs, uint64_t* len) {
  *len = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  hbam::Pipeline& p = ctx->f->pipe();
  hbam::SpanDev span;
  if (ctx->last_is_writables || (ctx->batch.n && !ctx->cursor.last_batch_span(&span))) {
    ctx->err = "hbam_encode_writables needs a one-window batch from hbam_decode_span";
    return HBAM_E_STATE;
  }
  uint64_t bytes = 0;
  int rc = ctx->batch.n ? p.encoded_bytes(span, &bytes) : HBAM_OK;
  if (rc != HBAM_OK) {
    ctx->err = p.error();
    return rc;
  }
  *len = bytes;
  if (offs) {  // encodings have the records' own lengths: record i starts where its bytes did
    const hadoop_bam::BatchView& h = ctx->batch;
    for (uint64_t i = 0; i < h.n; ++i) offs[i] = h.rest_off[i] - h.rest_off[0];
    offs[h.n] = bytes;
  }
  if (!out) return HBAM_OK;
  if (cap < bytes) {
    ctx->err = "output buffer too small for the encoded records";
    return HBAM_E_ARG;
  }
  if (bytes == 0) return HBAM_OK;
  hbam::DevBuf<uint8_t> dst(&p.streams());
  if (dst.reserve((bytes + 15) & ~15ull) != hipSuccess) {
    ctx->err = "hipMalloc failed";
    return HBAM_E_DEVICE;
  }
  rc = p.encode_writables(span, bytes, dst.p);
  if (rc != HBAM_OK) {
    ctx->err = p.error();
    return rc;
  }
  if (hipMemcpyAsync(out, dst.p, bytes, hipMemcpyDeviceToHost, p.stream()) != hipSuccess ||
      hipStreamSynchronize(p.stream()) != hipSuccess) {
    ctx->err = "hipMemcpy D2H failed";
    return HBAM_E_DEVICE;
  }
  return HBAM_OK;
}

int hbam_decode_writables(hbam_ctx* ctx, const void* buf, uint64_t len, const uint64_t* offs, uint64_t n,
                          hbam_batch* out) {
  memset(out, 0, sizeof *out);
  if (!ctx || (!ctx->f && !ctx->codec)) return HBAM_E_STATE;
  hbam::Pipeline& p = ctx->f ? ctx->f->pipe() : *ctx->codec;
  ctx->cursor.reset();
  ctx->last_is_writables = true;
  hbam::SpanDev& span = ctx->wspan;
  span = hbam::SpanDev();
  int rc = p.decode_writables(static_cast<const uint8_t*>(buf), len, offs, n, &span);
  if (rc != HBAM_OK) {
    ctx->err = p.error();
    span = hbam::SpanDev();
    return rc;
  }
  HostBatch& h = ctx->wbatch;
  h.n = 0;
  h.data_len = 0;
  h.window_pos.clear();
  ctx->batch = hadoop_bam::BatchView();
  rc = hadoop_bam::fetch_span(p, span, 0, span.n, &h, &ctx->err);
  if (rc != HBAM_OK) return rc;
  ctx->batch = hadoop_bam::BatchView::of(h);
  fill_batch(ctx->batch, out);
  out->status = span.status;
  if (span.status != HBAM_OK) {
    ctx->err = span.error;
    return span.status;
  }
  return HBAM_OK;
}

int hbam_build_splitting_index(hbam_ctx* ctx, int32_t granularity, uint8_t** buf, uint64_t* len) {
  *buf = nullptr;
  *len = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<uint8_t> out;
  int rc = SplittingBAMIndexer::index(*ctx->f, granularity, &out);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  *buf = static_cast<uint8_t*>(malloc(out.size() ? out.size() : 1));
  if (!*buf) return HBAM_E_NOMEM;
  memcpy(*buf, out.data(), out.size());
  *len = out.size();
  return HBAM_OK;
}

int hbam_splitting_entries(hbam_ctx* ctx, uint64_t vstart, uint64_t vend, int32_t granularity, uint64_t ordinal0,
                           uint64_t** entries, uint64_t* n_entries, uint64_t* n_records) {
  *entries = nullptr;
  *n_entries = *n_records = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<uint64_t> ent;
  int rc = SplittingBAMIndexer::entries(*ctx->f, vstart, vend, granularity, ordinal0, &ent, n_records);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  *entries = static_cast<uint64_t*>(malloc(ent.empty() ? 8 : ent.size() * 8));
  if (!*entries) return HBAM_E_NOMEM;
  if (!ent.empty()) memcpy(*entries, ent.data(), ent.size() * 8);
  *n_entries = ent.size();
  return HBAM_OK;
}

int hbam_splitting_index_for_records(const hbam_opts* opts, const uint64_t* voffs, uint64_t n, int32_t granularity,
                                     uint64_t file_size, uint8_t** buf, uint64_t* len) {
  *buf = nullptr;
  *len = 0;
  if (granularity <= 0) {
    g_open_err = "Granularity must be a positive integer";
    return HBAM_E_ARG;
  }
  hbam_opts o{};
  if (opts) o = *opts;
  if (o.device < 0 || o.device >= hbam_device_count()) {
    g_open_err = "no HIP device " + std::to_string(o.device);
    return HBAM_E_DEVICE;
  }
  // processAlignment (SplittingBAMIndexer.java:197-202): record 0, then every
  // record whose ordinal + 1 is a multiple of g; finish writes size << 16
  hbam::Pipeline p(o.device);
  if (!p.error().empty()) {
    g_open_err = p.error();
    return HBAM_E_DEVICE;
  }
  hbam::DevBuf<uint64_t> dv(&p.streams());
  std::vector<uint64_t> ent;
  hbam::SpanDev span;
  if (n) {
    if (dv.reserve(n) != hipSuccess || hipMemcpy(dv.p, voffs, n * 8, hipMemcpyHostToDevice) != hipSuccess) {
      g_open_err = "device buffer for the voffs";
      return HBAM_E_DEVICE;
    }
    span.n = n;
    span.rec_voff = dv.p;
    int rc = p.splitting_entries(span, (uint32_t)granularity, 0, &ent);
    if (rc != HBAM_OK) {
      g_open_err = p.error();
      return rc;
    }
  }
  std::vector<uint64_t> all;
  if (n) all.push_back(voffs[0]);
  if (granularity == 1 && n) ent.erase(ent.begin());  // record 0 is written once
  all.insert(all.end(), ent.begin(), ent.end());
  all.push_back(file_size << 16);
  *len = all.size() * 8;
  *buf = static_cast<uint8_t*>(malloc(*len));
  if (!*buf) return HBAM_E_NOMEM;
  for (size_t i = 0; i < all.size(); ++i)
    for (int b = 0; b < 8; ++b) (*buf)[8 * i + b] = (uint8_t)(all[i] >> (56 - 8 * b));
  return HBAM_OK;
}

int hbam_guess_record_starts(hbam_ctx* ctx, const uint64_t* begs, const uint64_t* ends, uint64_t n, uint64_t* out) {
  return hbam_guess_record_starts_hdr(ctx, -1, begs, ends, n, out);
}

int hbam_guess_record_starts_hdr(hbam_ctx* ctx, int32_t header_n_ref, const uint64_t* begs, const uint64_t* ends,
                                 uint64_t n, uint64_t* out) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<uint64_t> b(begs, begs + n), e(ends, ends + n), r;
  hadoop_bam::BAMSplitGuesser g(*ctx->f, header_n_ref);
  int rc = g.guessNextBAMRecordStarts(b, e, &r);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  if (n) memcpy(out, r.data(), n * 8);
  return HBAM_OK;
}

int hbam_guess_bgzf_block_starts(hbam_ctx* ctx, const uint64_t* begs, const uint64_t* ends, uint64_t n,
                                 uint64_t* out) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<uint64_t> b(begs, begs + n), e(ends, ends + n), r;
  int rc = hadoop_bam::guess_bgzf_batch(*ctx->f, b, e, &r, &ctx->err);
  if (rc != HBAM_OK) return rc;
  if (n) memcpy(out, r.data(), n * 8);
  return HBAM_OK;
}

int hbam_get_splits(hbam_ctx* ctx, const uint64_t* starts, const uint64_t* lengths, uint64_t n, const uint8_t* sbi,
                    uint64_t sbi_len, uint64_t* vstarts, uint64_t* vends, uint64_t* nout) {
  return hbam_get_splits_bai(ctx, starts, lengths, n, sbi, sbi_len, nullptr, 0, vstarts, vends, nout);
}

int hbam_get_splits_bai(hbam_ctx* ctx, const uint64_t* starts, const uint64_t* lengths, uint64_t n,
                        const uint8_t* sbi, uint64_t sbi_len, const uint8_t* bai, uint64_t bai_len, uint64_t* vstarts,
                        uint64_t* vends, uint64_t* nout) {
  *nout = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<FileSplit> sp(n);
  for (uint64_t i = 0; i < n; ++i) {
    sp[i].path = "bam";
    sp[i].start = starts[i];
    sp[i].length = lengths[i];
  }
  std::vector<FileVirtualSplit> out;
  int rc = BAMInputFormat::getSplits(*ctx->f, sp, sbi, sbi_len, &out, bai, bai_len);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  for (size_t i = 0; i < out.size(); ++i) {
    vstarts[i] = out[i].vStart;
    vends[i] = out[i].vEnd;
  }
  *nout = out.size();
  return HBAM_OK;
}

int hbam_blocks(hbam_ctx* ctx, uint64_t* coff, uint32_t* csize, uint32_t* isize, uint64_t* ustart, uint64_t cap,
                uint64_t* n) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  const std::vector<hbam::BlockInfo>* B = nullptr;
  int rc = ctx->f->all_blocks(&B);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  *n = B->size();
  for (size_t i = 0; i < B->size() && i < cap; ++i) {
    if (coff) coff[i] = (*B)[i].coff;
    if (csize) csize[i] = (*B)[i].csize;
    if (isize) isize[i] = (*B)[i].isize;
    if (ustart) ustart[i] = (*B)[i].ustart;
  }
  return HBAM_OK;
}

int hbam_read_inflated(hbam_ctx* ctx, uint64_t pos, uint64_t len, uint8_t* dst) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->cursor.reset();
  std::vector<uint8_t> v;
  int rc = ctx->f->read_inflated(pos, len, &v);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  if (v.size() != len) {
    ctx->err = "range beyond the inflated stream";
    return HBAM_E_ARG;
  }
  if (len) memcpy(dst, v.data(), len);
  return HBAM_OK;
}

int64_t hbam_get_key0(int32_t ref_idx, int32_t alignment_start0) {
  return BAMRecordReader::getKey0(ref_idx, alignment_start0);
}
int64_t hbam_get_key(int32_t ref_idx, int32_t alignment_start) {
  return BAMRecordReader::getKey(ref_idx, alignment_start);
}
int64_t hbam_murmurhash3(const void* key, uint64_t len, int32_t seed) {
  return hadoop_bam::murmurhash3(static_cast<const uint8_t*>(key), len, seed);
}

// ---- device-resident decode --------------------------------------------------
int32_t hbam_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int hbam_gpu_create(int32_t device, hbam_gpu** out) {
  *out = nullptr;
  int n = hbam_device_count();
  if (device < 0 || device >= n) {
    g_open_err = "no HIP device " + std::to_string(device);
    return HBAM_E_DEVICE;
  }
  auto* g = new hbam_gpu();
  g->device = device;
  *out = g;
  return HBAM_OK;
}

void hbam_gpu_destroy(hbam_gpu* g) { delete g; }

const char* hbam_gpu_error(hbam_gpu* g) { return g ? g->err.c_str() : g_open_err.c_str(); }

int hbam_gpu_load(hbam_gpu* g, const void* data, uint64_t len) {
  OpenOptions o;
  o.device = g->device;
  o.window_bytes = g->window;
  g->enc.release();  // owned by the old file's pipeline streams
  g->enc.owner = nullptr;
  g->f.reset();
  g->span = hbam::SpanDev();
  std::string err;
  int rc = BamFile::open_device_copy(static_cast<const uint8_t*>(data), len, o, &g->f, &err);
  if (rc != HBAM_OK) g->err = err;
  return rc;
}

int hbam_gpu_set_window(hbam_gpu* g, uint64_t window_bytes) {
  g->window = window_bytes ? window_bytes : hadoop_bam::kDefaultWindowBytes;
  if (g->f) g->f->set_window_bytes(g->window);
  return HBAM_OK;
}

int hbam_gpu_run(hbam_gpu* g, int32_t flags, hbam_gpu_stats* st) {
  memset(st, 0, sizeof *st);
  if (!g->f) {
    g->err = "hbam_gpu_run needs a loaded file";
    return HBAM_E_STATE;
  }
  return decode_device(*g->f, g->f->first_record_voff(), ~0ull, flags, st, &g->span, &g->err);
}

int hbam_gpu_index(hbam_gpu* g, int32_t granularity, uint8_t** buf, uint64_t* len, float* ms) {
  *buf = nullptr;
  *len = 0;
  *ms = 0;
  if (!g->f) return HBAM_E_STATE;
  hbam::Pipeline& p = g->f->pipe();
  p.timing = false;
  g->f->invalidate_window();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, p.stream());
  std::vector<uint8_t> out;
  int rc = SplittingBAMIndexer::index(*g->f, granularity, &out);
  (void)hipEventRecord(e1, p.stream());
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  g->span = hbam::SpanDev();
  if (rc != HBAM_OK) {
    g->err = g->f->error();
    return rc;
  }
  *buf = static_cast<uint8_t*>(malloc(out.size() ? out.size() : 1));
  if (!*buf) return HBAM_E_NOMEM;
  memcpy(*buf, out.data(), out.size());
  *len = out.size();
  return HBAM_OK;
}

int hbam_gpu_run_streamed(hbam_gpu* g, const void* data, uint64_t len, uint64_t piece_bytes, hbam_gpu_stats* st) {
  memset(st, 0, sizeof *st);
  if (!g->f || len != g->f->file_size()) {
    g->err = "hbam_gpu_run_streamed needs the loaded file's bytes";
    return HBAM_E_STATE;
  }
  hbam::Pipeline& p = g->f->pipe();
  p.timing = false;
  g->f->invalidate_window();
  // one window holding the whole file in the pipeline's own buffer (untimed)
  int rc = p.load(static_cast<const uint8_t*>(data), len, 0, true);
  if (rc != HBAM_OK) {
    g->err = p.error();
    return rc;
  }
  const uint64_t il0 = p.inflate_launches();
  g->span = hbam::SpanDev();
  // first record: the header end (the same position the resident pass starts at)
  std::unique_ptr<BamFile>& f = g->f;
  rc = p.locate();
  uint64_t first_pos = 0;
  if (rc == HBAM_OK) {
    const int64_t fp = p.pos_of_voff(f->first_record_voff());
    if (fp < 0) rc = HBAM_E_STATE;
    first_pos = (uint64_t)std::max<int64_t>(fp, 0);
  }
  if (rc == HBAM_OK)
    rc = p.run_streamed(static_cast<const uint8_t*>(data), len, piece_bytes, first_pos, &g->span, &st->ms_total);
  g->f->invalidate_window();
  if (rc != HBAM_OK) {
    g->err = p.error();
    st->status = rc;
    return rc;
  }
  st->n_blocks = p.blocks().size();
  st->compressed_bytes = p.file_len();
  st->inflated_bytes = p.total_u();
  st->records = g->span.n;
  st->status = g->span.status;
  st->windows = 1;
  st->inflate_launches = (int32_t)(p.inflate_launches() - il0);
  if (g->span.n) {
    (void)hipMemcpy(&st->first_voff, g->span.rec_voff, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&st->last_voff, g->span.rec_voff + g->span.n - 1, 8, hipMemcpyDeviceToHost);
  }
  if (g->span.status != HBAM_OK) g->err = g->span.error;
  return g->span.status;
}

void* hbam_host_alloc(uint64_t bytes) {
  // the library's page-locked blocks: on the current device's NUMA node (hbam_mem.cpp)
  void* p = nullptr;
  size_t got = 0;
  if (hbam::pinned_alloc(&p, bytes ? bytes : 1, &got) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(host_alloc_mu());
  host_allocs()[p] = got;
  return p;
}

void hbam_host_free(void* p) {
  if (!p) return;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> lk(host_alloc_mu());
    auto it = host_allocs().find(p);
    if (it == host_allocs().end()) return;
    bytes = it->second;
    host_allocs().erase(it);
  }
  hbam::pinned_free(p, bytes);
}

int hbam_gpu_reload(hbam_gpu* g, const void* data, uint64_t len, int32_t pinned, float* ms) {
  *ms = 0;
  if (!g->f) return HBAM_E_STATE;
  hbam::Pipeline& p = g->f->pipe();
  g->f->invalidate_window();
  int rc = p.load(static_cast<const uint8_t*>(data), len, 0, true);  // the copy target (untimed)
  if (rc == HBAM_OK) rc = p.reload(static_cast<const uint8_t*>(data), len, pinned != 0, ms);
  if (rc != HBAM_OK) g->err = p.error();
  g->span = hbam::SpanDev();
  return rc;
}

int hbam_gpu_d2d_bandwidth(hbam_gpu* g, uint64_t bytes, int32_t iters, float* gbps) {
  if (!g->f) return HBAM_E_STATE;
  int rc = g->f->pipe().d2d_bandwidth(bytes, iters, gbps);
  if (rc != HBAM_OK) g->err = g->f->pipe().error();
  return rc;
}

int hbam_gpu_encode_writables(hbam_gpu* g, int32_t iters, float* ms_per_iter, uint64_t* bytes) {
  *ms_per_iter = 0;
  *bytes = 0;
  if (!g->f) return HBAM_E_STATE;
  hbam::Pipeline& p = g->f->pipe();
  uint64_t nb = 0;
  g->enc.owner = &p.streams();
  int rc = p.encoded_bytes(g->span, &nb);
  if (rc != HBAM_OK) {
    g->err = p.error();
    return rc;
  }
  if (g->enc.reserve((nb + 15) & ~15ull) != hipSuccess) {
    g->err = "hipMalloc failed";
    return HBAM_E_DEVICE;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  rc = p.encode_writables(g->span, nb, g->enc.p);  // warm-up (also checks the launch)
  if (rc == HBAM_OK) {
    (void)hipEventRecord(e0, p.stream());
    for (int32_t i = 0; i < iters && rc == HBAM_OK; ++i) rc = p.encode_writables(g->span, nb, g->enc.p);
    (void)hipEventRecord(e1, p.stream());
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    *ms_per_iter = iters > 0 ? ms / (float)iters : 0.f;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc != HBAM_OK) {
    g->err = p.error();
    return rc;
  }
  g->enc_bytes = nb;
  *bytes = nb;
  return HBAM_OK;
}

int hbam_gpu_fetch_encoded(hbam_gpu* g, uint64_t pos, uint64_t len, uint8_t* dst) {
  if (pos > g->enc_bytes || len > g->enc_bytes - pos) {
    g->err = "range outside the encoded records";
    return HBAM_E_ARG;
  }
  if (len && hipMemcpy(dst, g->enc.p + pos, len, hipMemcpyDeviceToHost) != hipSuccess) return HBAM_E_DEVICE;
  return HBAM_OK;
}

int hbam_gpu_bgzf_compress(hbam_gpu* g, int32_t level, int32_t flags, int32_t iters, float* ms_per_iter,
                           uint64_t* out_len) {
  *ms_per_iter = 0;
  *out_len = 0;
  if (!g->f) return HBAM_E_STATE;
  hbam::Pipeline& p = g->f->pipe();
  if (!p.d_u() || p.base() != 0 || !p.at_eof() || p.blocks().empty()) {
    g->err = "hbam_gpu_bgzf_compress needs a one-window run (inflated stream) first";
    return HBAM_E_STATE;
  }
  std::vector<uint64_t> ustart;
  std::vector<uint32_t> lens;
  const auto& B = p.blocks();
  // the input's EOF terminator is re-added by HBAM_BGZF_EOF, not recompressed
  size_t nb = B.size();
  if ((flags & HBAM_BGZF_EOF) && nb && B[nb - 1].isize == 0) --nb;
  for (size_t i = 0; i < nb; ++i) {
    ustart.push_back(B[i].ustart);
    lens.push_back(B[i].isize);
  }
  // the run inflated the blocks from the first record on; the header's too
  int rc0 = p.inflate(0, (uint32_t)B.size());
  if (rc0 != HBAM_OK) {
    g->err = p.error();
    return rc0;
  }
  if (!g->bgzf) g->bgzf.reset(new hbam::BgzfCompressor(p.device()));
  float ms = 0, tot = 0;
  int rc = g->bgzf->compress(p.d_u(), ustart, lens, level, (flags & HBAM_BGZF_EOF) != 0, p.stream(), &ms);
  for (int32_t i = 0; i < iters && rc == HBAM_OK; ++i) {
    rc = g->bgzf->compress(p.d_u(), ustart, lens, level, (flags & HBAM_BGZF_EOF) != 0, p.stream(), &ms);
    tot += ms;
  }
  if (rc != HBAM_OK) {
    g->err = g->bgzf->error();
    return rc;
  }
  *ms_per_iter = iters > 0 ? tot / (float)iters : ms;
  *out_len = g->bgzf->out_len();
  return HBAM_OK;
}

int hbam_gpu_fetch_compressed(hbam_gpu* g, uint64_t pos, uint64_t len, uint8_t* dst) {
  const uint64_t n = g->bgzf ? g->bgzf->out_len() : 0;
  if (pos > n || len > n - pos) {
    g->err = "range outside the compressed output";
    return HBAM_E_ARG;
  }
  if (len && hipMemcpy(dst, g->bgzf->d_out() + pos, len, hipMemcpyDeviceToHost) != hipSuccess) return HBAM_E_DEVICE;
  return HBAM_OK;
}

int hbam_gpu_fetch(hbam_gpu* g, int64_t* keys, uint64_t* voffs, uint64_t cap) {
  const uint64_t n = std::min<uint64_t>(cap, g->span.n);
  if (keys && n && g->span.col.key) {
    if (hipMemcpy(keys, g->span.col.key, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return HBAM_E_DEVICE;
  }
  if (voffs && n) {
    if (hipMemcpy(voffs, g->span.rec_voff, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return HBAM_E_DEVICE;
  }
  return HBAM_OK;
}

}  // extern "C"
