// hbam_abi.cpp -- extern "C" boundary (include/hbam.h) over the C++ mirror.
#include "../../include/hbam.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "hbam_deflate_api.h"
#include "hbam_host.h"

using hadoop_bam::BAMInputFormat;
using hadoop_bam::BamFile;
using hadoop_bam::BAMRecordReader;
using hadoop_bam::FileSplit;
using hadoop_bam::FileVirtualSplit;
using hadoop_bam::SplittingBAMIndexer;

struct hbam_ctx {
  std::unique_ptr<BamFile> f;
  std::unique_ptr<hbam::Pipeline> codec;  // hbam_open_codec: a pipeline with no file
  std::string err;
  BAMRecordReader::Host batch;
  hbam::SpanDev span;  // device result of the last hbam_decode_span (valid until the next call)
  std::string text;
};

struct hbam_gpu {
  std::unique_ptr<hbam::Pipeline> p;
  std::string err;
  uint64_t first_pos = 0;  // inflated-stream position of the first record
  hbam::SpanDev span;
  hbam::DevBuf<uint8_t> enc;  // hbam_gpu_encode_writables output
  uint64_t enc_bytes = 0;
  std::unique_ptr<hbam::BgzfCompressor> bgzf;  // hbam_gpu_bgzf_compress
};

namespace {
std::string g_open_err;

int open_common(const void* data, uint64_t len, const hbam_opts* opts, bool header, hbam_ctx** out) {
  *out = nullptr;
  hbam_opts o{};
  if (opts) o = *opts;
  auto* c = new hbam_ctx();
  std::string err;
  int rc = BamFile::open(static_cast<const uint8_t*>(data), len, o.device, header, o.check_crc != 0, &c->f, &err);
  if (rc != HBAM_OK) {
    g_open_err = err;
    c->err = err;
    *out = c;  // caller may read hbam_last_error, then must hbam_close
    return rc;
  }
  *out = c;
  return HBAM_OK;
}

bool read_file(const char* path, std::vector<uint8_t>* buf, std::string* err) {
  FILE* fp = fopen(path, "rb");
  if (!fp) {
    *err = std::string("cannot open ") + path;
    return false;
  }
  fseek(fp, 0, SEEK_END);
  long n = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  buf->resize(n > 0 ? (size_t)n : 0);
  size_t got = n > 0 ? fread(buf->data(), 1, (size_t)n, fp) : 0;
  fclose(fp);
  if ((long)got != n) {
    *err = std::string("short read on ") + path;
    return false;
  }
  return true;
}
}  // namespace

extern "C" {

int32_t hbam_abi_version(void) { return HBAM_ABI_VERSION; }

int hbam_open_mem(const void* data, uint64_t len, const hbam_opts* opts, hbam_ctx** out) {
  return open_common(data, len, opts, true, out);
}

int hbam_open_bgzf(const void* data, uint64_t len, const hbam_opts* opts, hbam_ctx** out) {
  return open_common(data, len, opts, false, out);
}

int hbam_open(const char* path, const hbam_opts* opts, hbam_ctx** out) {
  std::vector<uint8_t> buf;
  std::string err;
  if (!read_file(path, &buf, &err)) {
    *out = new hbam_ctx();
    (*out)->err = err;
    return HBAM_E_IO;
  }
  return open_common(buf.data(), buf.size(), opts, true, out);
}

void hbam_close(hbam_ctx* ctx) { delete ctx; }

const char* hbam_last_error(hbam_ctx* ctx) { return ctx ? ctx->err.c_str() : g_open_err.c_str(); }

void hbam_free(void* p) { free(p); }

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
  out->n_blocks = f.pipe().blocks().size();
  out->uncompressed_size = f.pipe().total_u();
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

namespace {
void fill_batch(hbam_ctx* ctx, const hbam::SpanDev& span, hbam_batch* out) {
  auto& h = ctx->batch;
  out->n = span.n;
  out->ref_id = h.ref_id.data();
  out->pos = h.pos.data();
  out->l_seq = h.l_seq.data();
  out->next_ref_id = h.next_ref_id.data();
  out->next_pos = h.next_pos.data();
  out->tlen = h.tlen.data();
  out->l_read_name = h.l_read_name.data();
  out->mapq = h.mapq.data();
  out->bin = h.bin.data();
  out->n_cigar = h.n_cigar.data();
  out->flag = h.flag.data();
  out->key = h.key.data();
  out->voff = h.voff.data();
  out->rest_off = h.rest_off.data();
  out->rest_len = h.rest_len.data();
  out->data = h.data.data();
  out->data_len = h.data.size();
  out->status = span.status;
}
}  // namespace

int hbam_decode_span(hbam_ctx* ctx, uint64_t vstart, uint64_t vend, hbam_batch* out) {
  memset(out, 0, sizeof *out);
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  ctx->span = hbam::SpanDev();
  hbam::SpanDev& span = ctx->span;
  int rc = ctx->f->pipe().decode_span(vstart, vend, hbam::kReader, true, &span);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->pipe().error();
    span = hbam::SpanDev();
    return rc;
  }
  rc = hadoop_bam::fetch_span(ctx->f->pipe(), span, &ctx->batch, &ctx->err);
  if (rc != HBAM_OK) return rc;
  fill_batch(ctx, span, out);
  if (span.status != HBAM_OK) {
    ctx->err = span.error;
    return span.status;
  }
  return HBAM_OK;
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
  const hbam::SpanDev& span = ctx->span;
  if (span.data) {
    ctx->err = "hbam_encode_writables needs a span from hbam_decode_span";
    return HBAM_E_STATE;
  }
  uint64_t bytes = 0;
  int rc = p.encoded_bytes(span, &bytes);
  if (rc != HBAM_OK) {
    ctx->err = p.error();
    return rc;
  }
  *len = bytes;
  if (offs) {  // encodings have the records' own lengths: record i starts where its bytes did
    for (uint64_t i = 0; i < span.n; ++i) offs[i] = ctx->batch.rest_off[i] - 36;
    offs[span.n] = bytes;
  }
  if (!out) return HBAM_OK;
  if (cap < bytes) {
    ctx->err = "output buffer too small for the encoded records";
    return HBAM_E_ARG;
  }
  if (bytes == 0) return HBAM_OK;
  hbam::DevBuf<uint8_t> dst;
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
  ctx->span = hbam::SpanDev();
  hbam::SpanDev& span = ctx->span;
  int rc = p.decode_writables(static_cast<const uint8_t*>(buf), len, offs, n, &span);
  if (rc != HBAM_OK) {
    ctx->err = p.error();
    span = hbam::SpanDev();
    return rc;
  }
  rc = hadoop_bam::fetch_span(p, span, &ctx->batch, &ctx->err);
  if (rc != HBAM_OK) return rc;
  fill_batch(ctx, span, out);
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

int hbam_guess_record_starts(hbam_ctx* ctx, const uint64_t* begs, const uint64_t* ends, uint64_t n, uint64_t* out) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  std::vector<uint64_t> b(begs, begs + n), e(ends, ends + n), r;
  hadoop_bam::BAMSplitGuesser g(*ctx->f);
  int rc = g.guessNextBAMRecordStarts(b, e, &r);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->error();
    return rc;
  }
  memcpy(out, r.data(), n * 8);
  return HBAM_OK;
}

int hbam_guess_bgzf_block_starts(hbam_ctx* ctx, const uint64_t* begs, const uint64_t* ends, uint64_t n,
                                 uint64_t* out) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  std::vector<uint64_t> b(begs, begs + n), e(ends, ends + n), r;
  int rc = hadoop_bam::guess_bgzf_batch(*ctx->f, b, e, &r, &ctx->err);
  if (rc != HBAM_OK) return rc;
  if (n) memcpy(out, r.data(), n * 8);
  return HBAM_OK;
}

int hbam_get_splits(hbam_ctx* ctx, const uint64_t* starts, const uint64_t* lengths, uint64_t n, const uint8_t* sbi,
                    uint64_t sbi_len, uint64_t* vstarts, uint64_t* vends, uint64_t* nout) {
  *nout = 0;
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  std::vector<FileSplit> sp(n);
  for (uint64_t i = 0; i < n; ++i) {
    sp[i].path = "bam";
    sp[i].start = starts[i];
    sp[i].length = lengths[i];
  }
  std::vector<FileVirtualSplit> out;
  int rc = BAMInputFormat::getSplits(*ctx->f, sp, sbi, sbi_len, &out);
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
  const auto& b = ctx->f->pipe().blocks();
  *n = b.size();
  for (size_t i = 0; i < b.size() && i < cap; ++i) {
    if (coff) coff[i] = b[i].coff;
    if (csize) csize[i] = b[i].csize;
    if (isize) isize[i] = b[i].isize;
    if (ustart) ustart[i] = b[i].ustart;
  }
  return HBAM_OK;
}

int hbam_read_inflated(hbam_ctx* ctx, uint64_t pos, uint64_t len, uint8_t* dst) {
  if (!ctx || !ctx->f) return HBAM_E_STATE;
  std::vector<uint8_t> v;
  int rc = ctx->f->pipe().read_stream(pos, len, &v);
  if (rc != HBAM_OK) {
    ctx->err = ctx->f->pipe().error();
    return rc;
  }
  if (v.size() != len) {
    ctx->err = "range beyond the inflated stream";
    return HBAM_E_ARG;
  }
  memcpy(dst, v.data(), len);
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

// ---- device-resident pipeline ------------------------------------------------
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
  g->p.reset(new hbam::Pipeline(device));
  if (!g->p->error().empty()) {
    g_open_err = g->p->error();
    delete g;
    return HBAM_E_DEVICE;
  }
  *out = g;
  return HBAM_OK;
}

void hbam_gpu_destroy(hbam_gpu* g) { delete g; }

const char* hbam_gpu_error(hbam_gpu* g) { return g ? g->err.c_str() : g_open_err.c_str(); }

int hbam_gpu_load(hbam_gpu* g, const void* data, uint64_t len, uint64_t base_offset, int32_t n_ref,
                  uint64_t first_pos) {
  int rc = g->p->load(static_cast<const uint8_t*>(data), len, base_offset);
  if (rc == HBAM_OK) rc = g->p->locate();
  if (rc != HBAM_OK) {
    g->err = g->p->error();
    return rc;
  }
  if (first_pos == UINT64_MAX) {
    // whole file: parse the header with the same GPU-backed reader
    std::unique_ptr<BamFile> tmp;
    std::string err;
    rc = BamFile::open(static_cast<const uint8_t*>(data), len, g->p->device(), true, false, &tmp, &err);
    if (rc != HBAM_OK) {
      g->err = err;
      return rc;
    }
    g->p->set_n_ref(tmp->n_ref());
    g->first_pos = tmp->header_end();
  } else {
    g->p->set_n_ref(n_ref);
    g->first_pos = first_pos;
  }
  return HBAM_OK;
}

int hbam_gpu_run(hbam_gpu* g, int32_t flags, hbam_gpu_stats* st) {
  memset(st, 0, sizeof *st);
  hbam::Pipeline& p = *g->p;
  p.timing = (flags & 1) != 0;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, p.stream());
  const uint64_t lf0 = p.link_fallbacks(), il0 = p.inflate_launches(), lr0 = p.link_rewalks();
  int rc = p.locate();
  if (rc == HBAM_OK) rc = p.inflate(0, (uint32_t)p.blocks().size(), true);
  float ms_inflate = p.times.inflate, ms_huff = p.times.huff, ms_lz = p.times.lz77;
  if (rc == HBAM_OK) {
    rc = p.decode_span(p.voff_of(g->first_pos), ~0ull, hbam::kReader, (flags & 2) == 0, &g->span);
  }
  (void)hipEventRecord(e1, p.stream());
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&st->ms_total, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
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
  st->link_fallbacks = (int32_t)(p.link_fallbacks() - lf0);
  st->inflate_launches = (int32_t)(p.inflate_launches() - il0);
  st->link_rewalks = (int32_t)(p.link_rewalks() - lr0);
  if (p.timing) {
    st->ms_locate = p.times.locate;
    st->ms_inflate = ms_inflate;
    st->ms_huff = ms_huff;
    st->ms_lz77 = ms_lz;
    st->ms_chain = p.times.chain;
    st->ms_decode = p.times.decode;
  }
  if (g->span.n) {
    (void)hipMemcpy(&st->first_voff, g->span.rec_voff, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&st->last_voff, g->span.rec_voff + g->span.n - 1, 8, hipMemcpyDeviceToHost);
  }
  if (g->span.status != HBAM_OK) g->err = g->span.error;
  return g->span.status;
}

int hbam_gpu_run_streamed(hbam_gpu* g, const void* data, uint64_t len, uint64_t piece_bytes, hbam_gpu_stats* st) {
  memset(st, 0, sizeof *st);
  hbam::Pipeline& p = *g->p;
  p.timing = false;
  const uint64_t il0 = p.inflate_launches();
  g->span = hbam::SpanDev();
  int rc = p.run_streamed(static_cast<const uint8_t*>(data), len, piece_bytes, g->first_pos, &g->span, &st->ms_total);
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
  st->inflate_launches = (int32_t)(p.inflate_launches() - il0);
  if (g->span.n) {
    (void)hipMemcpy(&st->first_voff, g->span.rec_voff, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&st->last_voff, g->span.rec_voff + g->span.n - 1, 8, hipMemcpyDeviceToHost);
  }
  if (g->span.status != HBAM_OK) g->err = g->span.error;
  return g->span.status;
}

void* hbam_host_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void hbam_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int hbam_gpu_reload(hbam_gpu* g, const void* data, uint64_t len, int32_t pinned, float* ms) {
  *ms = 0;
  int rc = g->p->reload(static_cast<const uint8_t*>(data), len, pinned != 0, ms);
  if (rc != HBAM_OK) g->err = g->p->error();
  return rc;
}

int hbam_gpu_d2d_bandwidth(hbam_gpu* g, uint64_t bytes, int32_t iters, float* gbps) {
  int rc = g->p->d2d_bandwidth(bytes, iters, gbps);
  if (rc != HBAM_OK) g->err = g->p->error();
  return rc;
}

int hbam_gpu_encode_writables(hbam_gpu* g, int32_t iters, float* ms_per_iter, uint64_t* bytes) {
  *ms_per_iter = 0;
  *bytes = 0;
  hbam::Pipeline& p = *g->p;
  uint64_t nb = 0;
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
  hbam::Pipeline& p = *g->p;
  if (!p.d_u()) {
    g->err = "hbam_gpu_bgzf_compress needs a run (inflated stream) first";
    return HBAM_E_STATE;
  }
  std::vector<uint64_t> ustart;
  std::vector<uint32_t> lens;
  for (const auto& b : p.blocks()) {
    ustart.push_back(b.ustart);
    lens.push_back(b.isize);
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
