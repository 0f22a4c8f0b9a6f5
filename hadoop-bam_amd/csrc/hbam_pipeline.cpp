// hbam_pipeline.cpp -- host orchestration of one HBM window of the gfx950 BAM
// read pipeline (see hbam_pipeline.h).
#include "hbam_pipeline.h"

#include <thread>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "hbam_launch.h"

namespace hbam {

namespace {
constexpr uint32_t kStreamInflateBlocks = 8192;  // run_streamed: blocks per inflate call
#ifndef HBAM_INFLATE_CHUNK
#define HBAM_INFLATE_CHUNK 65536
#endif
// blocks per phase-A/B launch pair: C2's 52 K blocks in one chunk beat two
// overlapped ones (phase B cannot share a CU with phase A, and each chunk pays
// its launch tails): 16.07-16.16 vs 16.13-16.25 ms per pass in three A/B runs
// (profiles/r06_late/variants_chunk_*.log); 20 K: 16.31, 16 K: -0.7 %, 8 K: -4 %
constexpr uint32_t kInflateChunkBlocks = HBAM_INFLATE_CHUNK;
constexpr int kMaxChainIters = 64;
constexpr int kMaxLinkFix = 4;        // re-walk rounds before the serial link
constexpr int kMaxFreeStarts = 64;    // header candidates tried by a free-start locate
// e_true of an open window: records may run past its last block
constexpr uint64_t kOpenEnd = 1ull << 62;
}  // namespace

hipError_t create_stream(hipStream_t* s, StreamLevel level) {
  if (level == StreamLevel::kNormal) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, level == StreamLevel::kHigh ? greatest : least);
}

Pipeline::Pipeline(int device) : device_(device) {
  if (hipSetDevice(device) != hipSuccess) {
    err_ = "hipSetDevice failed";
    return;
  }
  if (create_stream(&stream_, StreamLevel::kNormal) != hipSuccess ||
      create_stream(&stream_b_, StreamLevel::kNormal) != hipSuccess ||
      create_stream(&stream_t_, StreamLevel::kNormal) != hipSuccess ||
      create_stream(&stream_copy_, StreamLevel::kNormal) != hipSuccess ||
      create_stream(&stream_stage_, StreamLevel::kLow) != hipSuccess)
    err_ = "hipStreamCreate failed";
  streams_.s[0] = stream_;
  streams_.s[1] = stream_b_;
  streams_.s[2] = stream_t_;
  streams_.s[3] = stream_copy_;
  streams_.n = 4;
  // the staging copy (stage()) runs on its own stream, outside streams_: a
  // buffer of the decode that grows waits for the decode's streams only, not
  // for the next window's bytes on their way (that wait cost 5-13 ms per
  // drop-in window); stage_ itself is written there and read on stream_
  stage_owner_.s[0] = stream_stage_;
  stage_owner_.s[1] = stream_;
  stage_owner_.n = 2;
  stage_.owner = &stage_owner_;
  own(own_file_, own_spare_, dblocks_, ref_len_, du_, tokens_[0], tokens_[1], hout_, tables_[0], tables_[1],
      tinfo_[0], tinfo_[1], g_, x_, x2_, entry_, base_arr_, summary_, dead_, cand_, sorted_, isz_, ust_, cnt_, flags_,
      errv_, need_, rec_pos_, rec_voff_, rcand_, force_, wcnt_, counters_, list_, scan_tmp_, cols_, long_rec_,
      long_n_, wbuf_, woffs_, wbad_, scalars_, fuse_);
  for (auto& e : ev_) (void)hipEventCreate(&e);
  for (auto& e : sync_ev_) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : tab_ev_) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : hdone_ev_) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
}

Pipeline::~Pipeline() {
  if (stage_thr_.joinable()) stage_thr_.join();
  (void)hipSetDevice(device_);
  // this pipeline's own streams only: other contexts on the GPU run on
  (void)streams_.sync();
  (void)stage_owner_.sync();
  streams_.n = 0;  // drained: the member buffers release without waiting (the streams go below)
  stage_owner_.n = 0;
  if (rb_buf_) pinned_free(rb_buf_, rb_cap_);
  for (auto& e : ev_) (void)hipEventDestroy(e);
  for (auto& e : sync_ev_) (void)hipEventDestroy(e);
  for (auto& e : tab_ev_) (void)hipEventDestroy(e);
  for (auto& e : hdone_ev_) (void)hipEventDestroy(e);
  for (auto& e : tev_) (void)hipEventDestroy(e);
  for (auto& e : copy_ev_) (void)hipEventDestroy(e);
  for (hipStream_t s : {stream_b_, stream_t_, stream_copy_, stream_stage_, stream_})
    if (s) (void)hipStreamDestroy(s);
}

int Pipeline::fail(int code, const std::string& msg) {
  err_ = msg;
  return code;
}

int Pipeline::hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return kOk;
  err_ = std::string(what) + ": " + hipGetErrorString(e);
  return kErrDevice;
}

#define HIPCHK(expr)                                   \
  do {                                                 \
    int _rc = hip_check((expr), #expr);                \
    if (_rc != kOk) return _rc;                        \
  } while (0)

int Pipeline::load(const uint8_t* data, uint64_t len, uint64_t base, bool at_eof, uint64_t* host_bytes) {
  HostSource m;
  m.mem = data;
  m.size = len;
  return load_from(m, 0, len, base, at_eof, host_bytes);
}

int Pipeline::load(const HostSource& src, uint64_t len, uint64_t base, bool at_eof, uint64_t* host_bytes) {
  return load_from(src, base, len, base, at_eof, host_bytes);
}

int Pipeline::load_from(const HostSource& src, uint64_t src_off, uint64_t len, uint64_t base, bool at_eof,
                        uint64_t* host_bytes) {
  HIPCHK(hipSetDevice(device_));
  // dst <- file bytes [base + a, base + a + n) (src offset src_off + a)
  auto feed = [&](uint64_t a, uint64_t n) -> int {
    std::string e;
    const int rc = feed_load_.copy(dfile_ + a, src, src_off + a, n, stream_, &e);
    if (rc != kOk) err_ = e;
    return rc;
  };
  static const bool tr = getenv("HBAM_CURSOR_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  // the prefix of [base, base + len) that the window in place already holds
  uint64_t keep = 0;
  if (dfile_ && own_file_.p && dfile_ == own_file_.p + (base_ & 15) && base >= base_ && base < base_ + flen_)
    keep = std::min(base_ + flen_, base + len) - base;
  const uint8_t* old = keep ? dfile_ + (base - base_) : nullptr;
  if (keep) own_file_.swap(own_spare_);
  // byte `base` lands at a buffer offset of base % 16: the kernels address the
  // window in file coordinates (dfile_ - base_) with 16 B aligned loads
  HIPCHK(own_file_.reserve(len + 16 + kFilePad));
  dfile_ = own_file_.p + (base & 15);
  if (keep) HIPCHK(hipMemcpyAsync(dfile_, old, keep, hipMemcpyDeviceToDevice, stream_));
  uint64_t host = 0;
  if (len > keep) {
    // [a, b): the part of the new bytes a stage() copy already brought over
    const uint64_t a = std::max(base + keep, stage_lo_), b = std::min(base + len, stage_hi_);
    if (stage_hi_ > stage_lo_ && a < b) {
      if (int rc = stage_wait()) return rc;
      if (a > base + keep)
        if (int rc = feed(keep, a - base - keep)) return rc;
      HIPCHK(hipMemcpyAsync(dfile_ + (a - base), stage_.p + (a - stage_lo_), b - a, hipMemcpyDeviceToDevice, stream_));
      if (base + len > b)
        if (int rc = feed(b - base, base + len - b)) return rc;
      host = len - keep - (b - a);
    } else {
      if (int rc = feed(keep, len - keep)) return rc;
      host = len - keep;
    }
  }
  if (host_bytes) *host_bytes = host;
  HIPCHK(hipMemsetAsync(dfile_ + len, 0, kFilePad, stream_));
  HIPCHK(rb_sync(stream_));
  if (tr)
    fprintf(stderr, "[load] %.3f ms: %llu B kept, %llu B from host\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
            (unsigned long long)keep, (unsigned long long)host);
  flen_ = len;
  base_ = base;
  at_eof_ = at_eof;
  window_end_ = base + len;
  hblocks_.clear();
  inflated_.clear();
  total_u_ = 0;
  return kOk;
}

hipError_t Pipeline::rb(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  // every read, a counter as the block table, goes through k_readback into
  // page-locked memory: a D2H copy into pageable memory waits behind other
  // copies on the DMA engines (a drop-in batch's columns: the 4-byte candidate
  // count of a window's locate took 13 ms behind them)
  hipError_t e;
  if (rb_stream_ && rb_stream_ != s && (e = rb_sync(rb_stream_)) != hipSuccess) return e;
  size_t off = (rb_used_ + 15) & ~size_t(15);
  if (off + bytes > rb_cap_) {
    if (!rb_items_.empty() && (e = rb_sync(s)) != hipSuccess) return e;  // the old buffer drains first
    if (rb_buf_) pinned_free(rb_buf_, rb_cap_);
    rb_buf_ = nullptr;
    rb_cap_ = 0;
    void* q = nullptr;
    size_t got = 0;
    if ((e = pinned_alloc(&q, std::max<size_t>(bytes + 4096, 1 << 20), &got)) != hipSuccess) return e;
    rb_buf_ = static_cast<uint8_t*>(q);
    rb_cap_ = got;
    off = 0;
  }
  if ((e = launch_readback(rb_buf_ + off, src, bytes, s)) != hipSuccess) return e;
  rb_items_.push_back(RbItem{dst, off, bytes});
  rb_used_ = off + bytes;
  rb_stream_ = s;
  return hipSuccess;
}

hipError_t Pipeline::rb_sync(hipStream_t s) {
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess && rb_stream_ && rb_stream_ != s) e = hipStreamSynchronize(rb_stream_);
  if (e != hipSuccess) return e;
  for (const RbItem& it : rb_items_) memcpy(it.dst, rb_buf_ + it.off, it.bytes);
  rb_items_.clear();
  rb_used_ = 0;
  rb_stream_ = nullptr;
  return hipSuccess;
}

int Pipeline::copy_from_host(uint8_t* dst, const HostSource& src, uint64_t off, uint64_t len) {
  HIPCHK(hipSetDevice(device_));
  std::string e;
  const int rc = feed_load_.copy(dst, src, off, len, stream_, &e);
  if (rc != kOk) {
    HIPCHK(rb_sync(stream_));  // pieces already queued land before the caller moves on
    return fail(rc, e);
  }
  HIPCHK(rb_sync(stream_));
  return kOk;
}

int Pipeline::stage_wait() {
  if (stage_thr_.joinable()) stage_thr_.join();
  const int rc = stage_rc_;
  stage_rc_ = kOk;
  if (rc != kOk) {
    stage_lo_ = stage_hi_ = 0;
    return fail(rc, "staged host->HBM copy: " + stage_msg_);
  }
  return kOk;
}

int Pipeline::reserve_stage(uint64_t bytes) {
  HIPCHK(hipSetDevice(device_));
  if (int rc = stage_wait()) return rc;
  HIPCHK(stage_.reserve(bytes));
  return kOk;
}

int Pipeline::stage(const HostSource& src, uint64_t lo, uint64_t hi) {
  HIPCHK(hipSetDevice(device_));
  if (hi <= lo || (lo == stage_lo_ && hi == stage_hi_)) return kOk;  // nothing new to stage
  if (int rc = stage_wait()) return rc;
  HIPCHK(stage_.reserve(hi - lo));  // growing it waits for the device
  // A copy from pageable memory (the mapped file) returns only when it is
  // done, so a helper thread issues it: the caller goes on queueing this
  // window's decode while the next window's bytes cross the link.
  uint8_t* dst = stage_.p;
  const int dev = device_;
  hipStream_t cs = stream_stage_;
  const HostSource* hs = &src;
  stage_thr_ = std::thread([this, dst, hs, lo, hi, dev, cs]() {
    std::string msg;
    hipError_t e = hipSetDevice(dev);
    int rc = e == hipSuccess ? feed_stage_.copy(dst, *hs, lo, hi - lo, cs, &msg) : (int)kErrDevice;
    if (rc == kOk && (e = hipStreamSynchronize(cs)) != hipSuccess) rc = kErrDevice;
    if (rc == kErrDevice && msg.empty()) msg = hipGetErrorString(e);
    if (rc != kOk) (void)hipStreamSynchronize(cs);  // pieces already queued land first
    stage_msg_ = msg;
    stage_rc_ = rc;
  });
  stage_lo_ = lo;
  stage_hi_ = hi;
  return kOk;
}

int Pipeline::attach_device(const uint8_t* dptr, uint64_t len, uint64_t base, bool at_eof) {
  if ((reinterpret_cast<uintptr_t>(dptr) - base) & 15)
    return fail(kErrArg, "attach_device: file offset and device address differ in 16 B alignment");
  dfile_ = const_cast<uint8_t*>(dptr);
  flen_ = len;
  base_ = base;
  at_eof_ = at_eof;
  window_end_ = base + len;
  hblocks_.clear();
  inflated_.clear();
  total_u_ = 0;
  return kOk;
}

int Pipeline::reload(const uint8_t* data, uint64_t len, bool pinned, float* ms) {
  if (!dfile_ || dfile_ != own_file_.p + (base_ & 15) || len != flen_)
    return fail(kErrState, "reload needs a loaded window of the same size");
  HIPCHK(hipSetDevice(device_));
  uint8_t* staging = nullptr;
  if (pinned && len) {  // page-locked copy of the bytes (untimed), as a JNI direct buffer would be
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&staging), len, hipHostMallocDefault));
    memcpy(staging, data, len);
  }
  auto body = [&]() -> int {
    HIPCHK(hipEventRecord(ev_[6], stream_));
    if (len) HIPCHK(hipMemcpyAsync(dfile_, staging ? staging : data, len, hipMemcpyHostToDevice, stream_));
    HIPCHK(hipEventRecord(ev_[7], stream_));
    HIPCHK(hipEventSynchronize(ev_[7]));
    HIPCHK(hipEventElapsedTime(ms, ev_[6], ev_[7]));
    return kOk;
  };
  const int rc = body();
  if (staging) (void)hipHostFree(staging);
  return rc;
}

int Pipeline::d2d_bandwidth(uint64_t bytes, int iters, float* gbps) {
  *gbps = 0;
  DevBuf<uint8_t> a(&streams_), b(&streams_);
  HIPCHK(a.reserve(bytes));
  HIPCHK(b.reserve(bytes));
  HIPCHK(hipMemsetAsync(a.p, 1, bytes, stream_));
  HIPCHK(hipMemcpyAsync(b.p, a.p, bytes, hipMemcpyDeviceToDevice, stream_));  // warm-up
  HIPCHK(hipEventRecord(ev_[6], stream_));
  for (int i = 0; i < iters; ++i) HIPCHK(hipMemcpyAsync(b.p, a.p, bytes, hipMemcpyDeviceToDevice, stream_));
  HIPCHK(hipEventRecord(ev_[7], stream_));
  HIPCHK(hipEventSynchronize(ev_[7]));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, ev_[6], ev_[7]));
  *gbps = (float)(2.0 * (double)bytes * iters / ((double)ms * 1e6));  // read + write
  return kOk;
}

int Pipeline::inflate_tokens(uint64_t* n) {
  *n = 0;
  const size_t nb = hblocks_.size();
  if (nb == 0) return kOk;
  std::vector<HuffOut> h(nb);
  HIPCHK(hipStreamSynchronize(stream_));
  HIPCHK(hipStreamSynchronize(stream_b_));
  HIPCHK(hipMemcpy(h.data(), hout_.p, nb * sizeof(HuffOut), hipMemcpyDeviceToHost));
  for (const HuffOut& o : h) *n += o.ntok;
  return kOk;
}

int Pipeline::set_ref_lengths(const std::vector<int32_t>& lens) {
  HIPCHK(ref_len_.reserve(lens.size() + 1));
  if (!lens.empty())
    HIPCHK(hipMemcpyAsync(ref_len_.p, lens.data(), lens.size() * 4, hipMemcpyHostToDevice, stream_));
  HIPCHK(rb_sync(stream_));
  n_ref_len_ = (uint32_t)lens.size();
  return kOk;
}

int Pipeline::locate_range(uint64_t lo, uint64_t hi, bool partial, bool free_start, uint32_t nprev, uint64_t ubase,
                           hipStream_t s, uint32_t* nnew, uint64_t* tail) {
  *nnew = 0;
  *tail = hi;
  const uint8_t* fbase = dfile_ - base_;  // absolute file coordinates
  const uint64_t len = hi - lo;
  // candidate capacity assumes >= 1 KiB per block on average; denser files
  // (or any chain break) take the serial walk, whose table bound is len/26.
  const uint32_t cap = (uint32_t)std::min<uint64_t>(len / 1024 + 4096, 0x7fffffffu);
  const uint32_t walk_cap = (uint32_t)std::min<uint64_t>(len / 26 + 16, 0x7fffffffu);
  HIPCHK(cand_.reserve(cap));
  HIPCHK(flags_.reserve(5));
  // {0, 0, 0xffffffff, 0, 0} by fill kernels: a small pageable H2D can wait
  // behind other contexts' or the drop-in batches' copies on the DMA engines
  HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags_.p), 0, 5, s));
  HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags_.p + 2), -1, 1, s));
  // flags_[0] = candidate count, [1] = chain break, [2] = first big ISIZE, [3] = cut tail,
  // [4] = empty blocks
  HIPCHK(launch_bgzf_scan(fbase, base_, lo, hi, cand_.p, cap, flags_.p, s));
  uint32_t count = 0;
  HIPCHK(rb(&count, flags_.p, 4, s));
  HIPCHK(rb_sync(s));
  bool serial = count > cap || (count == 0 && len > 0);
  if (free_start && count == 0) return kOk;  // no header in the window: no blocks
  uint32_t n = serial ? 0 : count;
  // the block table of n located blocks: ustart by a scan, read back in place
  // into page-locked hblocks_ (the read lands at the next rb_sync)
  auto queue_table = [&](uint32_t nt) -> int {
    HIPCHK(dblocks_.grow(nprev + nt + 1));
    HIPCHK(isz_.reserve(nt + 1));
    HIPCHK(ust_.reserve(nt + 1));
    size_t sb = 0;
    HIPCHK(launch_block_ustart(dblocks_.p + nprev, nt, isz_.p, ust_.p, nullptr, &sb, ubase, s));
    HIPCHK(scan_tmp_.reserve(sb + 16));
    HIPCHK(launch_block_ustart(dblocks_.p + nprev, nt, isz_.p, ust_.p, scan_tmp_.p, &sb, ubase, s));
    HIPCHK(hblocks_.resize(nprev + nt));
    if (nt) HIPCHK(launch_readback(hblocks_.data() + nprev, dblocks_.p + nprev, nt * sizeof(BlockInfo), s));
    return kOk;
  };
  std::vector<uint64_t> starts;  // free start: candidates to try, in order
  if (!serial && n > 0) {
    HIPCHK(dblocks_.grow(nprev + n + 1));
    HIPCHK(sorted_.reserve(n));
    size_t tmp_bytes = 0;
    HIPCHK(sort_u64(nullptr, &tmp_bytes, cand_.p, sorted_.p, n, s));
    HIPCHK(scan_tmp_.reserve(tmp_bytes + 16));
    HIPCHK(sort_u64(scan_tmp_.p, &tmp_bytes, cand_.p, sorted_.p, n, s));
    if (free_start) {
      starts.resize(std::min<uint32_t>(n, kMaxFreeStarts));
      HIPCHK(rb(starts.data(), sorted_.p, starts.size() * 8, s));
      HIPCHK(rb_sync(s));
      lo = starts[0];
    }
    HIPCHK(launch_bgzf_verify(fbase, lo, hi, sorted_.p, n, dblocks_.p + nprev, flags_.p + 1, partial ? 1u : 0u, s));
    uint32_t fl[4];
    uint64_t last = 0;
    HIPCHK(rb(fl, flags_.p + 1, 16, s));
    HIPCHK(rb(&last, sorted_.p + n - 1, 8, s));
    // the table queued behind the verdict as if the chain holds (a false
    // header candidate breaks it: the serial walk below then rebuilds the
    // table); a block cut by hi is the last entry, and the scan's entries
    // before it do not depend on it
    if (int rc = queue_table(n)) return rc;
    HIPCHK(rb_sync(s));
    if (!fl[0] && empty_blocks_ != kEmptyUnknown) empty_blocks_ += fl[3];
    if (fl[0]) serial = true;
    else if (fl[1] != 0xffffffffu) return fail(kErrFormat, "BGZF block with ISIZE > 65536 (unsupported on device)");
    else if (fl[2]) {  // the last candidate's block is cut by hi: next range
      n -= 1;
      *tail = last;
    }
    if (!serial) {
      HIPCHK(hblocks_.resize(nprev + n));  // (drops the cut block's entry)
      *nnew = n;
      return kOk;
    }
  }
  if (serial) {
    empty_blocks_ = kEmptyUnknown;  // (the walk does not count them)
    uint32_t out[4];
    HIPCHK(dblocks_.grow(nprev + walk_cap + 1));
    if (starts.empty()) starts.push_back(lo);
    bool found = false;
    for (size_t j = 0; j < starts.size() && !found; ++j) {
      HIPCHK(hipMemsetAsync(flags_.p, 0, 16, s));
      HIPCHK(launch_bgzf_walk(fbase, starts[j], hi, dblocks_.p + nprev, walk_cap, flags_.p, partial ? 1u : 0u, s));
      HIPCHK(rb(out, flags_.p, 16, s));
      HIPCHK(rb_sync(s));
      n = out[0];
      const uint64_t at = (uint64_t)out[2] | ((uint64_t)out[3] << 32);
      if (out[1] != kOk) {
        if (free_start) continue;  // a false header candidate: try the next one
        return fail((int)out[1], "malformed BGZF block at offset " + std::to_string(at));
      }
      if (free_start && n == 0) continue;
      if (partial) *tail = at;
      found = true;
    }
    if (!found) {
      if (free_start) return kOk;  // no block chain in the window
      return fail(kErrFormat, "malformed BGZF block");
    }
  }
  if (int rc = queue_table(n)) return rc;
  HIPCHK(rb_sync(s));
  *nnew = n;
  return kOk;
}

int Pipeline::finish_blocks() {
  const uint32_t n = (uint32_t)hblocks_.size();
  total_u_ = n ? hblocks_[n - 1].ustart + hblocks_[n - 1].isize : 0;
  HIPCHK(du_.grow(total_u_ + kUPad));
  HIPCHK(hipMemsetAsync(du_.p + total_u_, 0, kUPad, stream_));
  inflated_.resize(n, 0);
  HIPCHK(hout_.grow(n + 1));
  // dead positions: [htsjdk] an empty block right after an exhausted one.
  // The verify kernel counted the empty blocks: with none, or only the EOF
  // block at the end, no walk over the block table (1.7 MB for C2, read
  // while the GPU waits) is needed.
  std::vector<uint64_t> dead;
  if (empty_blocks_ == 1 && n >= 2 && hblocks_[n - 1].isize == 0) {
    dead.push_back(hblocks_[n - 1].ustart);
  } else if (empty_blocks_ != 0) {
    for (uint32_t k = 1; k < n; ++k)
      if (hblocks_[k].isize == 0 && (dead.empty() || dead.back() != hblocks_[k].ustart))
        dead.push_back(hblocks_[k].ustart);
  }
  HIPCHK(dead_.reserve(dead.size() + 1));
  // from page-locked memory by a copy kernel: no host wait before the
  // inflate is planned (hdead_ is rewritten only by the next locate, after
  // its own read-backs have synchronized stream_)
  HIPCHK(hdead_.resize(dead.size()));
  if (!dead.empty()) {
    memcpy(hdead_.data(), dead.data(), dead.size() * 8);
    HIPCHK(launch_readback(dead_.p, hdead_.data(), dead.size() * 8, stream_));
  }
  ndead_ = (uint32_t)dead.size();
  return kOk;
}

int Pipeline::locate(bool free_start) {
  HIPCHK(hipSetDevice(device_));
  if (timing) HIPCHK(hipEventRecord(ev_[0], stream_));
  hblocks_.clear();
  inflated_.clear();
  empty_blocks_ = 0;
  uint32_t n = 0;
  uint64_t tail = 0;
  int rc = locate_range(base_, base_ + flen_, !at_eof_, free_start, 0, 0, stream_, &n, &tail);
  if (rc != kOk) return rc;
  window_end_ = at_eof_ ? base_ + flen_ : tail;
  if (n && at_eof_ && free_start) window_end_ = hblocks_[n - 1].coff + hblocks_[n - 1].csize;
  if (timing) {
    HIPCHK(hipEventRecord(ev_[1], stream_));
    HIPCHK(hipEventSynchronize(ev_[1]));
    (void)hipEventElapsedTime(&times.locate, ev_[0], ev_[1]);
  }
  return finish_blocks();
}

int Pipeline::run_streamed(const uint8_t* data, uint64_t len, uint64_t piece, uint64_t first_pos, SpanDev* out,
                           float* ms) {
  *ms = 0;
  *out = SpanDev();
  if (!dfile_ || dfile_ != own_file_.p || len != flen_ || base_ != 0 || !at_eof_)
    return fail(kErrState, "run_streamed needs the whole file loaded in one window");
  HIPCHK(hipSetDevice(device_));
  if (int rc = stage_wait()) return rc;  // no staged copy in flight over the window being replaced
  piece = std::max<uint64_t>(piece, 1ull << 20);
  const uint64_t np = std::max<uint64_t>(1, (len + piece - 1) / piece);
  // capacity up front, so that nothing reallocates under queued work (grow()
  // still handles a file that outruns the estimates, at the cost of a wait)
  HIPCHK(dblocks_.grow(len / 16384 + 4096));
  HIPCHK(hout_.grow(len / 16384 + 4096));
  HIPCHK(du_.grow(std::max<uint64_t>(total_u_, 4 * len) + kUPad));
  const uint64_t chunk_u = std::min<uint64_t>(8 * piece, (uint64_t)kInflateChunkBlocks * 65536);
  for (int i = 0; i < 2; ++i) HIPCHK(tokens_[i].reserve(chunk_u + 16));
  for (int i = 0; i < 2; ++i) {
    HIPCHK(tables_[i].reserve((uint64_t)kInflateChunkBlocks * kHuffTableImage));
    HIPCHK(tinfo_[i].reserve(kInflateChunkBlocks));
  }
  HIPCHK(streams_.sync());

  // Piece k's copy and its locate run in order on stream_copy_, the inflate
  // of located blocks on the inflate streams.  (With locate on its own stream,
  // which shares a hardware queue with stream_ at GPU_MAX_HW_QUEUES = 4, every
  // locate waited behind the queued inflates: copy and decode serialized.)
  auto queue_copy = [&](uint64_t k) -> int {
    const uint64_t o = k * piece, sz = std::min(piece, len - o);
    HIPCHK(hipMemcpyAsync(dfile_ + o, data + o, sz, hipMemcpyHostToDevice, stream_copy_));
    return kOk;
  };
  HIPCHK(hipEventRecord(ev_[6], stream_copy_));
  if (int rc0 = queue_copy(0)) return rc0;
  hblocks_.clear();
  inflated_.clear();
  empty_blocks_ = 0;
  total_u_ = 0;
  uint64_t lo = base_;
  uint32_t nb = 0, queued = 0;  // blocks located / handed to inflate
  for (uint64_t k = 0; k < np; ++k) {
    const bool last = k + 1 == np;
    const uint64_t hi = base_ + (last ? len : (k + 1) * piece);
    uint32_t nnew = 0;
    uint64_t tail = hi;
    int rc = locate_range(lo, hi, !last, false, nb, total_u_, stream_copy_, &nnew, &tail);
    if (rc != kOk) return rc;
    if (!last && (rc = queue_copy(k + 1)) != kOk) return rc;  // on the wire while piece k inflates
    if (nnew) {
      const BlockInfo& e = hblocks_[nb + nnew - 1];
      total_u_ = e.ustart + e.isize;
      HIPCHK(du_.grow(total_u_ + kUPad));
      HIPCHK(hout_.grow(nb + nnew + 1));
      inflated_.resize(nb + nnew, 0);
      nb += nnew;
    }
    // inflate in launches of >= kStreamInflateBlocks blocks: a piece's few
    // thousand blocks alone would leave most CUs idle in each round's tail
    if (nb > queued && (nb - queued >= kStreamInflateBlocks || last)) {
      rc = inflate(queued, nb, true, false, false);  // (phase B beside the next piece's phase A)
      if (rc != kOk) return rc;
      queued = nb;
    }
    lo = tail;
  }
  window_end_ = base_ + len;
  int rc = finish_blocks();  // (the inflates: ordered before stream_'s next work)
  if (rc != kOk) return rc;
  HIPCHK(flags_.reserve(4));
  const uint32_t none = 0xffffffffu;
  uint32_t first = none;
  HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags_.p + 3), (int)none, 1, stream_));
  HIPCHK(launch_first_error_hout(hout_.p, 0, nb, flags_.p + 3, stream_));
  HIPCHK(rb(&first, flags_.p + 3, 4, stream_));
  HIPCHK(rb_sync(stream_));
  if (first != none) {
    HuffOut ho;
    HIPCHK(rb(&ho, hout_.p + first, sizeof ho, stream_));
    HIPCHK(rb_sync(stream_));
    std::fill(inflated_.begin(), inflated_.end(), 0);
    const char* what = ho.status == kErrFormat ? "Did not inflate expected amount" : "invalid DEFLATE data";
    return fail(ho.status, std::string(what) + " in BGZF block at offset " + std::to_string(hblocks_[first].coff));
  }
  rc = decode_span(voff_of(first_pos), ~0ull, kReader, true, out);
  if (rc != kOk) return rc;
  HIPCHK(hipEventRecord(ev_[7], stream_));
  HIPCHK(hipEventSynchronize(ev_[7]));
  HIPCHK(hipEventElapsedTime(ms, ev_[6], ev_[7]));
  return kOk;
}

int Pipeline::inflate(uint32_t b0, uint32_t b1, bool force, bool check, bool join) {
  HIPCHK(hipSetDevice(device_));
  inflate_queued_ = false;
  const uint32_t nblk = (uint32_t)hblocks_.size();
  b1 = std::min(b1, nblk);
  if (b0 >= b1) return kOk;
  const uint8_t* fbase = dfile_ - base_;
  if (timing) HIPCHK(hipEventRecord(ev_[2], stream_));
  // Chunks of up to kInflateChunkBlocks blocks: per chunk the table build and
  // phase A in rounds, then phase B.  Production runs overlap them: phase A
  // on stream_, phase B on stream_b_ after it, the round-0 tables of chunk j
  // on stream_t_ beside phase A of chunk j-1, token and table buffers by
  // chunk parity (~0.7 ms per C2 pass faster than one stream).  A timed run
  // (measurement) puts every launch on stream_, each bracketed by events, so
  // its per-kernel times are kernel durations, as rocprofv3 reports them.
  const bool serial = timing;
  hipStream_t sB = serial ? stream_ : stream_b_, sT = serial ? stream_ : stream_t_;
  struct Chunk { uint32_t b, e; };
  std::vector<Chunk> chunks;
  // (the GPU is idle here: the common case -- nothing of [b0, b1) inflated
  // yet -- is planned without a walk over the blocks)
  const bool fresh = force || std::find(inflated_.begin() + b0, inflated_.begin() + b1, (uint8_t)1) ==
                                  inflated_.begin() + b1;
  uint32_t b = b0;
  while (b < b1) {
    if (!fresh && inflated_[b]) { ++b; continue; }
    // even chunks (a short last chunk would pay a whole wave tail for few blocks)
    const uint32_t left = b1 - b;
    const uint32_t nchunks = (left + kInflateChunkBlocks - 1) / kInflateChunkBlocks;
    const uint32_t per = (left + nchunks - 1) / nchunks;
    uint32_t e = b;
    if (fresh) e = std::min(b1, b + per);
    else while (e < b1 && e - b < per && !inflated_[e]) ++e;
    chunks.push_back({b, e});
    b = e;
  }
  const bool any = !chunks.empty();
  const size_t nc = chunks.size();
  const size_t per_chunk = 2 * (2 * kInflateRounds + 1);  // event pairs: tables + phase A per round, phase B
  if (timing && tev_.size() < per_chunk * nc) {
    const size_t old = tev_.size();
    tev_.resize(per_chunk * nc);
    for (size_t i = old; i < tev_.size(); ++i) HIPCHK(hipEventCreate(&tev_[i]));
  }
  // size every buffer up front: a reallocation inside the loop could free a
  // token buffer that phase B of an earlier chunk is still reading
  uint64_t max_u = 64, max_nb = 0;
  for (const Chunk& c : chunks) {
    max_u = std::max(max_u, hblocks_[c.e - 1].ustart + hblocks_[c.e - 1].isize - hblocks_[c.b].ustart);
    max_nb = std::max<uint64_t>(max_nb, c.e - c.b);
  }
  const int nbuf = nc > 1 && !serial ? 2 : 1;
  if (any) {
    for (int i = 0; i < nbuf; ++i) {
      HIPCHK(tokens_[i].reserve(max_u + 16));  // phase B reads tokens as uint4
      HIPCHK(tables_[i].reserve(max_nb * kHuffTableImage));
      HIPCHK(tinfo_[i].reserve(max_nb));
    }
    if (!serial) {  // phase B and the table builds see everything queued on stream_ before this call
      HIPCHK(hipEventRecord(sync_ev_[0], stream_));
      HIPCHK(hipStreamWaitEvent(stream_b_, sync_ev_[0], 0));
      HIPCHK(hipStreamWaitEvent(stream_t_, sync_ev_[0], 0));
    }
  }
  size_t ne = 0;  // events recorded (serial)
  auto mark = [&]() -> hipError_t { return serial ? hipEventRecord(tev_[ne++], stream_) : hipSuccess; };
  for (size_t j = 0; j < nc; ++j) {
    const uint32_t cb = chunks[j].b, ce = chunks[j].e;
    const int par = serial ? 0 : (int)(j & 1);
    const uint64_t cu = hblocks_[cb].ustart;
    if (!serial && j >= 2) {
      HIPCHK(hipStreamWaitEvent(stream_, sync_ev_[2 + par], 0));  // B(j-2) released the token buffer
      HIPCHK(hipStreamWaitEvent(stream_t_, hdone_ev_[par], 0));   // A(j-2) released the table buffer
    }
    // rounds: each decode stops a block before its next DEFLATE header, which
    // the next round's table build parses (the last round decodes inline)
    // (the first chunk's round-0 tables run on stream_ itself: nothing runs
    // beside them, and a cross-stream wait costs ~15 us at the pass's start)
    const bool t_own = !serial && j > 0;
    for (uint32_t r = 0; r < kInflateRounds; ++r) {
      HIPCHK(mark());
      HIPCHK(launch_huff_tables(fbase, dblocks_.p, cb, ce - cb, tables_[par].p, tinfo_[par].p, hout_.p, r,
                                r == 0 && t_own ? sT : stream_));
      HIPCHK(mark());
      if (r == 0 && t_own) {
        HIPCHK(hipEventRecord(tab_ev_[par], stream_t_));
        HIPCHK(hipStreamWaitEvent(stream_, tab_ev_[par], 0));
      }
      HIPCHK(mark());
      HIPCHK(launch_inflate_huff_prebuilt(fbase, dblocks_.p, cb, ce - cb, cu, tokens_[par].p, hout_.p,
                                          tables_[par].p, tinfo_[par].p, r, r + 1 < kInflateRounds ? 1u : 0u,
                                          stream_));
      HIPCHK(mark());
    }
    // the last chunk's phase B on stream_ itself: nothing of this call is
    // left to overlap it, and the chain after it then needs no cross-stream wait
    const bool b_own = !serial && (j + 1 < nc || !join);
    hipStream_t sBj = b_own ? sB : stream_;
    if (!serial) HIPCHK(hipEventRecord(hdone_ev_[par], stream_));
    if (b_own) {
      HIPCHK(hipEventRecord(sync_ev_[par], stream_));
      HIPCHK(hipStreamWaitEvent(stream_b_, sync_ev_[par], 0));
    }
    HIPCHK(mark());
    HIPCHK(launch_inflate_lz77(dblocks_.p, cb, ce - cb, cu, tokens_[par].p, hout_.p, du_.p, sBj));
    HIPCHK(mark());
    if (!serial) HIPCHK(hipEventRecord(sync_ev_[2 + par], sBj));
    std::fill(inflated_.begin() + cb, inflated_.begin() + ce, (uint8_t)1);
    ++inflate_launches_;
  }
  if (any && !serial) {  // everything after this call on stream_ sees phase B done
    if (!join) HIPCHK(hipStreamWaitEvent(stream_, sync_ev_[2 + ((nc - 1) & 1)], 0));  // (with join it ran on stream_)
    if (nc >= 2) HIPCHK(hipStreamWaitEvent(stream_, sync_ev_[2 + ((nc - 2) & 1)], 0));
  }
  float tab_ms = 0, huff_ms = 0, lz_ms = 0;
  if (timing && any) {
    HIPCHK(hipEventSynchronize(tev_[ne - 1]));
    for (size_t i = 0; i < ne; i += 2) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, tev_[i], tev_[i + 1]);
      const size_t k = (i / 2) % (2 * kInflateRounds + 1);  // position of the pair within its chunk
      (k == 2 * kInflateRounds ? lz_ms : (k & 1) ? huff_ms : tab_ms) += ms;
    }
  }
  if (!any) {
    times.inflate = times.huff = times.lz77 = times.tables = 0;
    return kOk;
  }
  inflate_queued_ = true;
  if (!check) return kOk;  // the caller checks hout_ once all blocks are queued
  HIPCHK(queue_inflate_check(b0, b1));
  if (timing) HIPCHK(hipEventRecord(ev_[3], stream_));
  HIPCHK(rb_sync(stream_));
  if (timing) {
    (void)hipEventElapsedTime(&times.inflate, ev_[2], ev_[3]);
    times.tables = tab_ms;
    times.huff = huff_ms;
    times.lz77 = lz_ms;
  }
  return inflate_verdict(b0, b1);
}

hipError_t Pipeline::queue_inflate_check(uint32_t b0, uint32_t b1) {
  hipError_t e = flags_.reserve(4);
  if (e == hipSuccess) e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags_.p + 3), -1, 1, stream_);
  if (e == hipSuccess) e = launch_first_error_hout(hout_.p, b0, b1 - b0, flags_.p + 3, stream_);
  infl_first_ = 0xffffffffu;
  if (e == hipSuccess) e = rb(&infl_first_, flags_.p + 3, 4, stream_);
  return e;
}

int Pipeline::inflate_verdict(uint32_t b0, uint32_t b1) {
  const uint32_t first = infl_first_;
  if (first == 0xffffffffu) return kOk;
  HuffOut ho;
  HIPCHK(rb(&ho, hout_.p + b0 + first, sizeof ho, stream_));
  HIPCHK(rb_sync(stream_));
  for (uint32_t k = b0; k < b1; ++k) inflated_[k] = 0;
  const BlockInfo& bad = hblocks_[b0 + first];
  const char* what = ho.status == kErrFormat ? "Did not inflate expected amount" : "invalid DEFLATE data";
  return fail(ho.status, std::string(what) + " in BGZF block at offset " + std::to_string(bad.coff));
}

uint32_t Pipeline::block_containing(uint64_t pos) const {
  // first block with ustart + isize > pos (non-empty block containing pos)
  uint32_t lo = 0, hi = (uint32_t)hblocks_.size();
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (hblocks_[mid].ustart + hblocks_[mid].isize > pos) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// [htsjdk] BlockCompressedInputStream.getFilePointer normalization.
uint64_t Pipeline::voff_of(uint64_t pos) const {
  const uint32_t n = (uint32_t)hblocks_.size();
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (hblocks_[mid].ustart >= pos) hi = mid; else lo = mid + 1;
  }
  if (lo < n && hblocks_[lo].ustart == pos) return hblocks_[lo].coff << 16;
  if (lo == 0) return base_ << 16;
  const BlockInfo& b = hblocks_[lo - 1];
  if (pos - b.ustart < b.isize) return (b.coff << 16) | (pos - b.ustart);
  return (b.coff + b.csize) << 16;
}

int64_t Pipeline::pos_of_voff(uint64_t voff) const {
  const uint64_t coff = voff >> 16, uoff = voff & 0xffff;
  const uint32_t n = (uint32_t)hblocks_.size();
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (hblocks_[mid].coff >= coff) hi = mid; else lo = mid + 1;
  }
  if (lo >= n) return (coff == window_end_ && uoff == 0) ? (int64_t)total_u_ : -1;
  if (hblocks_[lo].coff != coff || uoff > hblocks_[lo].isize) return -1;
  return (int64_t)(hblocks_[lo].ustart + uoff);
}

// Smallest position q with voff_of(q) >= vend (voffs increase with q).
uint64_t Pipeline::q_end_of(uint64_t vend) const {
  const uint64_t c = vend >> 16, u = vend & 0xffff;
  const uint32_t n = (uint32_t)hblocks_.size();
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (hblocks_[mid].coff >= c) hi = mid; else lo = mid + 1;
  }
  if (lo >= n) return total_u_ + 1;  // every position of the window qualifies
  const BlockInfo& b = hblocks_[lo];
  if (b.coff == c) return b.ustart + std::min<uint64_t>(u, b.isize);
  return b.ustart;
}

int Pipeline::read_stream(uint64_t pos, uint64_t len, std::vector<uint8_t>* out) {
  out->clear();
  if (pos >= total_u_) return kOk;
  len = std::min(len, total_u_ - pos);
  uint32_t b0 = block_containing(pos), b1 = block_containing(pos + len - 1) + 1;
  int rc = inflate(b0, b1);
  if (rc != kOk) return rc;
  out->resize(len);
  HIPCHK(rb(out->data(), du_.p + pos, len, stream_));
  HIPCHK(rb_sync(stream_));
  return kOk;
}

int Pipeline::decode_span(uint64_t vstart, uint64_t vend, ChainMode mode, bool decode, SpanDev* out) {
  *out = SpanDev();
  const int64_t sp = pos_of_voff(vstart);
  if (sp < 0) return fail(kErrIO, "Invalid file pointer: " + std::to_string(vstart));
  return decode_span_pos((uint64_t)sp, vend, mode, decode, out);
}

int Pipeline::decode_span_pos(uint64_t p0, uint64_t vend, ChainMode mode, bool decode, SpanDev* out) {
  HIPCHK(hipSetDevice(device_));
  *out = SpanDev();
  const uint64_t q_end = q_end_of(vend);
  out->p0 = p0;
  out->q_end = q_end;
  out->next_pos = p0;
  const uint32_t nblk = (uint32_t)hblocks_.size();
  if (p0 >= q_end || p0 >= total_u_) return kOk;
  const uint32_t k0 = block_containing(p0);
  uint32_t k1 = std::min(nblk, block_containing(std::min(q_end, total_u_) - 1) + 1);
  uint32_t inf_end = std::min(nblk, k1 + 2);
  ChainArgs a{};
  a.blocks = dblocks_.p;
  a.e_true = at_eof_ ? total_u_ : kOpenEnd;
  a.p0 = p0;
  a.q_end = q_end;
  a.dead = dead_.p;
  a.ndead = ndead_;
  a.n_ref = n_ref_;
  a.k0 = k0;
  a.validate = mode != kReader ? 0 : stringency_ == kStrict ? 2 : stringency_ == kLenient ? 1 : 0;
  a.ref_len = n_ref_len_ == (uint32_t)std::max(n_ref_, 0) && n_ref_len_ ? ref_len_.p : nullptr;
  if (timing) HIPCHK(hipEventRecord(ev_[0], stream_));
  float infl_ms = 0, huff_ms = 0, lz_ms = 0, tab_ms = 0;
  bool lists = true;  // chain v2 lists hold every record start (no overflow)
  const bool dec = decode && mode == kReader;
  Columns c{};
  // the list path: check + output in one launch (k_rec_check_out); its results
  bool fused = false;
  uint64_t fused_total = 0;
  uint32_t fused_first = 0xffffffffu;
  // the span's tail (deferred long keys + the next record's start) queued
  // with k_rec_check_out, gated on its verdict, read back with it
  bool spec_tail = false;
  uint64_t spec_next = 0, spec_voff[2] = {0, 0};
  for (int it = 0;; ++it) {
    if (it >= kMaxChainIters) return fail(kErrState, "record chain did not converge");
    after_stop_pending_ = false;  // (only the last iteration's stop counts)
    // production runs check the inflate's DEFLATE status with the link
    // check's read-back (one host round trip fewer; the chain kernels take
    // any bytes, and their results are not used before the verdict)
    const bool defer = !timing;
    int rc = inflate(k0, inf_end, false, !defer);
    bool check_pending = false;
    if (rc == kOk && defer && inflate_queued_) {
      HIPCHK(queue_inflate_check(k0, inf_end));
      check_pending = true;
    }
    if (timing) {
      infl_ms += times.inflate;
      huff_ms += times.huff;
      lz_ms += times.lz77;
      tab_ms += times.tables;
    }
    if (rc != kOk) return rc;
    a.u = du_.p;
    a.e_inf = inf_end < nblk ? hblocks_[inf_end].ustart : total_u_;
    a.k1 = k1;
    const uint32_t nb = k1 - k0;
    HIPCHK(g_.reserve(nb));
    HIPCHK(x_.reserve(nb));
    HIPCHK(x2_.reserve(nb));
    HIPCHK(entry_.reserve(nb));
    HIPCHK(summary_.reserve(4));
    HIPCHK(cnt_.reserve(nb + 1));
    HIPCHK(errv_.reserve(nb + 1));
    HIPCHK(need_.reserve(1));
    HIPCHK(rcand_.reserve(nb));
    HIPCHK(force_.reserve(nb));
    HIPCHK(wcnt_.reserve(nb));
    HIPCHK(list_.reserve((uint64_t)nb * kListCap));
    HIPCHK(base_arr_.reserve(nb + 1));
    HIPCHK(counters_.reserve(4));
    size_t lsb = 0;
    HIPCHK(link_scan_bytes(nb, &lsb));
    HIPCHK(scan_tmp_.reserve(lsb + 16));
    a.g = g_.p;
    a.x = x_.p;
    a.x2 = x2_.p;
    a.entry = entry_.p;
    a.summary = summary_.p;
    a.cnt = cnt_.p;
    a.err = errv_.p;
    a.need = need_.p;
    a.cand = rcand_.p;
    a.force = force_.p;
    a.wcnt = wcnt_.p;
    a.list = list_.p;
    a.counters = counters_.p;
    a.base = base_arr_.p;
    a.scan_tmp = scan_tmp_.p;
    a.scan_bytes = lsb;
    HIPCHK(hipMemsetAsync(need_.p, 0, 8, stream_));
    HIPCHK(hipMemsetAsync(counters_.p, 0, 16, stream_));
    HIPCHK(launch_chain(a, mode, kStageWalk, stream_));  // candidates + lane-per-block walks
    // link: max-scan of the walk exits; re-walk blocks that are off the chain
    bool serial = false;
    // HBAM_CURSOR_TRACE: the blocks the link check left off the chain
    auto dump_off_chain = [&]() {
      if (!getenv("HBAM_CURSOR_TRACE")) return;
      std::vector<uint64_t> fv(nb), gv(nb), xv(nb), ev(nb), inv(nb);
      (void)hipStreamSynchronize(stream_);
      (void)hipMemcpy(fv.data(), force_.p, nb * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(gv.data(), g_.p, nb * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(xv.data(), x_.p, nb * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(ev.data(), entry_.p, nb * 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(inv.data(), base_arr_.p, nb * 8, hipMemcpyDeviceToHost);
      for (uint32_t i = 0, shown = 0; i < nb && shown < 8; ++i) {
      if (fv[i] == ~0ull) continue;
      const BlockInfo& b = hblocks_[a.k0 + i];
      fprintf(stderr, "[chain]   block %u (of %u) ustart %llu end %llu: force %llx g %llx x %llx in %llx entry %llx\n",
                i, nb, (unsigned long long)b.ustart, (unsigned long long)(b.ustart + b.isize),
                (unsigned long long)fv[i], (unsigned long long)gv[i], (unsigned long long)xv[i],
                (unsigned long long)inv[i], (unsigned long long)ev[i]);
      ++shown;
      }
    };
    uint64_t sm[2] = {0, 0};
    unsigned long long need = 0;
    // the lists' record counts scanned into base_arr_ (the output offsets of
    // k_rec_check_out; their total bounds the span's records) and the list
    // overflow flag come back with the chain's end in one host round trip
    HIPCHK(fuse_.reserve(4));
    uint64_t bound = 0, last_base = 0;
    uint32_t ovf = 0, last_cnt = 0;
    auto list_bound = [&]() -> hipError_t {
      hipError_t e = launch_list_counts(a, stream_);
      size_t tb = 0;
      if (e == hipSuccess) e = scan_u32_to_u64(nullptr, &tb, cnt_.p, base_arr_.p, nb, stream_);
      if (e == hipSuccess) e = scan_tmp_.reserve(tb + 16);
      a.scan_tmp = scan_tmp_.p;  // (a grown buffer serves the next link check too)
      if (e == hipSuccess) e = scan_u32_to_u64(scan_tmp_.p, &tb, cnt_.p, base_arr_.p, nb, stream_);
      if (e == hipSuccess) e = rb(&last_base, base_arr_.p + nb - 1, 8, stream_);
      if (e == hipSuccess) e = rb(&last_cnt, cnt_.p + nb - 1, 4, stream_);
      if (e == hipSuccess) e = rb(&ovf, counters_.p + 2, 4, stream_);
      return e;
    };
    // the chain's end: the link max-scan's last entry (read before
    // list_bound's scan overwrites base_arr_) and the last block's exit
    uint64_t t[2] = {0, 0};
    auto chain_end = [&]() -> hipError_t {
      hipError_t e = rb(&t[0], base_arr_.p + nb - 1, 8, stream_);
      if (e == hipSuccess) e = rb(&t[1], x2_.p + nb - 1, 8, stream_);
      return e;
    };
    bool spec_bound = false;  // chain end + list bound read with the first link check
    bool early_zeroed = false;  // k_rec_check_out's counters zeroed with them
    for (int fix = 0;; ++fix) {
      HIPCHK(hipMemsetAsync(counters_.p, 0, 8, stream_));
      HIPCHK(launch_chain(a, mode, kStageLinkCheck, stream_));
      uint32_t ctr[2] = {0, 0};
      HIPCHK(rb(ctr, counters_.p, 8, stream_));
      // first round: queue the chain end and the list bound as if the link
      // holds (it does in every production pass: link_rewalks 0); a re-walk
      // or the serial link recomputes them
      const bool spec = fix == 0 && !timing;
      if (spec) {
        HIPCHK(chain_end());
        HIPCHK(list_bound());
        // k_rec_check_out's counters too (they do not depend on the bound):
        // after the host wait only its launch remains
        HIPCHK(long_n_.reserve(1));
        HIPCHK(hipMemsetAsync(long_n_.p, 0, 4, stream_));
        HIPCHK(hipMemsetAsync(fuse_.p, 0xff, 12, stream_));  // early-stop key, first failing block: none
        early_zeroed = true;
      }
      HIPCHK(rb_sync(stream_));
      if (check_pending) {
        check_pending = false;
        if (int vr = inflate_verdict(k0, inf_end)) return vr;
      }
      if (spec && ctr[0] == 0 && ctr[1] == 0) {
        spec_bound = true;
        break;
      }
      if (ctr[0] || (ctr[1] && fix == kMaxLinkFix)) {
        if (getenv("HBAM_CURSOR_TRACE"))
          fprintf(stderr, "[chain] serial link: blocks [%u, %u) e_inf %llu e_true %llu p0 %llu rewalk round %d, "
                  "%u blocks off the chain, serial request %u\n", a.k0, a.k1, (unsigned long long)a.e_inf,
                  (unsigned long long)a.e_true, (unsigned long long)a.p0, fix, ctr[1], ctr[0]);
        dump_off_chain();
        serial = true;
        break;
      }
      if (ctr[1] == 0) break;
      if (getenv("HBAM_CURSOR_TRACE")) {
        fprintf(stderr, "[chain] rewalk round %d: %u blocks off the chain\n", fix, ctr[1]);
        dump_off_chain();
      }
      ++link_rewalks_;
      HIPCHK(launch_chain(a, mode, kStageRewalk, stream_));
    }
    if (serial) {  // exact serial link (writes entry[] + summary), then lists off entry[]
      ++link_fallbacks_;
      HIPCHK(launch_chain(a, mode, kStageSerialLink, stream_));
      HIPCHK(launch_chain(a, mode, kStageRewalkAll, stream_));
      HIPCHK(rb(sm, summary_.p, 16, stream_));
      HIPCHK(list_bound());
      HIPCHK(rb_sync(stream_));
    } else {  // final chain position = max of every walk exit; no stop
      if (!spec_bound) {
        HIPCHK(chain_end());
        HIPCHK(list_bound());
        HIPCHK(rb_sync(stream_));
      }
      sm[0] = nb == 1 ? t[1] : std::max(t[0], t[1]);
      sm[1] = 0;
    }
    bound = last_base + last_cnt;
    lists = ovf == 0;
    // a list overflowed (indexer mode: records shorter than 36 bytes): the
    // per-block walks count and emit the records instead (k_rec_count,
    // k_rec_emit)
    fused = lists;
    if (!lists) ++record_fallbacks_;
    if (fused) {
      // outputs sized by the lists' records, then check + positions + voffs +
      // fields + keys in one launch, each block at its scanned list offset
      HIPCHK(rec_pos_.reserve(bound + 1));
      HIPCHK(rec_voff_.reserve(bound + 1));
      if (dec) {
        int rc = alloc_columns(bound, total_u_, &c, !early_zeroed);
        if (rc != kOk) return rc;
      }
      if (!early_zeroed) HIPCHK(hipMemsetAsync(fuse_.p, 0xff, 12, stream_));  // early-stop key, first failing block: none
      a.fuse_bad = reinterpret_cast<uint64_t*>(fuse_.p);
      a.fuse_flags = fuse_.p + 2;
      a.rec_pos = rec_pos_.p;
      a.rec_voff = rec_voff_.p;
      if (timing) HIPCHK(hipEventRecord(ev_[1], stream_));
      HIPCHK(launch_rec_check_out(a, mode, dec, c, bound + 1, stream_));
      const bool spec = !timing;
      if (spec) {
        const unsigned long long* gb = reinterpret_cast<const unsigned long long*>(fuse_.p);
        if (dec) HIPCHK(launch_long_hash(du_.p, rec_pos_.p, c, stream_, gb, need_.p, a.e_inf));
        HIPCHK(scalars_.reserve(8));
        HIPCHK(launch_next_pos(du_.p, rec_pos_.p, bound, p0, mode, scalars_.p, stream_, gb, need_.p, a.e_inf));
        HIPCHK(rb(&spec_next, scalars_.p, 8, stream_));
        if (bound) {  // (stale unless the gate opens: then unused)
          HIPCHK(rb(&spec_voff[0], rec_voff_.p, 8, stream_));
          HIPCHK(rb(&spec_voff[1], rec_voff_.p + bound - 1, 8, stream_));
        }
      }
      uint64_t bad = 0;
      uint32_t fl[2] = {0, 0};
      HIPCHK(rb(&need, need_.p, 8, stream_));
      HIPCHK(rb(&bad, fuse_.p, 8, stream_));
      HIPCHK(rb(fl, fuse_.p + 2, 4, stream_));
      HIPCHK(rb_sync(stream_));
      spec_tail = spec && bad == ~0ull && need <= a.e_inf;
      fused_first = fl[0];
      if (bad == ~0ull) {
        fused_total = bound;  // every block kept its whole list
      } else {
        // the span ends at the first block that stops: its records stand at
        // their final offsets, later blocks' records lie past them and are
        // dropped, and that block's status (if any) is the span's -- a
        // failure in a later block is never reached (k_rec_check_out)
        const uint64_t k = bad >> kFusedBadShift;
        fused_total = bad & ((1ull << kFusedBadShift) - 1);
        if (fl[0] != k) fused_first = 0xffffffffu;
        // (diagnostic) records listed after the stop, which it drops: read
        // with the span's last readback, no round trip of its own
        HIPCHK(hipMemsetAsync(fuse_.p + 3, 0, 4, stream_));
        HIPCHK(launch_records_after(cnt_.p, nb, (uint32_t)k, fuse_.p + 3, stream_));
        HIPCHK(rb(&after_stop_flag_, fuse_.p + 3, 4, stream_));
        after_stop_pending_ = true;
      }
    } else {
      HIPCHK(launch_chain(a, mode, kStageCount, stream_));  // count + validate by walking
      HIPCHK(rb(&need, need_.p, 8, stream_));
      HIPCHK(rb_sync(stream_));
    }
    const uint64_t final_pos = sm[0];
    const bool stopped = sm[1] != 0;
    if (need > a.e_inf && inf_end < nblk) {  // a record needs bytes beyond the inflated range
      inf_end = std::min(nblk, block_containing(std::min<uint64_t>(need, total_u_) - 1) + 2);
      continue;
    }
    if (stopped && final_pos + 36 > a.e_inf && inf_end < nblk) {
      inf_end = std::min(nblk, inf_end + 4);
      continue;
    }
    if (!stopped && final_pos < q_end && final_pos < total_u_ && k1 < nblk && final_pos >= hblocks_[k1].ustart) {
      k1 = std::min(nblk, block_containing(std::min(final_pos, q_end - 1)) + 1);
      inf_end = std::max(inf_end, std::min(nblk, k1 + 2));
      continue;
    }
    break;
  }
  const uint32_t nb = k1 - k0;
  // first failing block: records before it stand, later blocks are dropped
  const uint32_t none = 0xffffffffu;
  uint32_t first = fused_first;
  if (!fused) {
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flags_.p + 3), (int)none, 1, stream_));
    HIPCHK(launch_first_error_i32(errv_.p, nb, flags_.p + 3, stream_));
    HIPCHK(rb(&first, flags_.p + 3, 4, stream_));
    HIPCHK(rb_sync(stream_));
  }
  int32_t code = 0;
  if (first != none) {
    HIPCHK(rb(&code, errv_.p + first, 4, stream_));
    HIPCHK(rb_sync(stream_));
    // (k_rec_count) the first block that stops, with or without an error:
    // the iteration ends there
    if (!fused) HIPCHK(launch_truncate_counts(cnt_.p, nb, flags_.p + 3, stream_));
  }
  if (first != none && code != kStopClean) {
    out->status = code;
    const BlockInfo& b = hblocks_[k0 + first];
    const char* what = code == kErrFormat ? "Invalid record (SAMFormatException)"
                       : code == kErrTrunc ? "Premature EOF in BAM record"
                       : code == kErrArg   ? "Reference index not found in sequence dictionary"
                                           : "Invalid alignment";
    out->error = std::string(what) + " (BGZF block at offset " + std::to_string(b.coff) + ")";
  }
  uint64_t total = fused_total;
  if (!fused) {
    HIPCHK(base_arr_.reserve(nb + 1));
    size_t tb = 0;
    HIPCHK(scan_u32_to_u64(nullptr, &tb, cnt_.p, base_arr_.p, nb, stream_));
    HIPCHK(scan_tmp_.reserve(tb + 16));
    HIPCHK(scan_u32_to_u64(scan_tmp_.p, &tb, cnt_.p, base_arr_.p, nb, stream_));
    uint64_t last_base = 0;
    uint32_t last_cnt = 0;
    HIPCHK(rb(&last_base, base_arr_.p + nb - 1, 8, stream_));
    HIPCHK(rb(&last_cnt, cnt_.p + nb - 1, 4, stream_));
    HIPCHK(rb_sync(stream_));
    total = last_base + last_cnt;
    HIPCHK(rec_pos_.reserve(total + 1));
    HIPCHK(rec_voff_.reserve(total + 1));
    a.base = base_arr_.p;
    a.rec_pos = rec_pos_.p;
    a.rec_voff = rec_voff_.p;
    if (dec) {
      int rc = alloc_columns(total, total_u_, &c);
      if (rc != kOk) return rc;
    }
  }
  out->n = total;
  out->rec_pos = rec_pos_.p;
  out->rec_voff = rec_voff_.p;
  if (dec) out->col = c;
  if (!fused) {  // a block listed more starts than kListCap: per-block walks
    HIPCHK(launch_chain(a, mode, kStageEmit, stream_));
    if (timing) HIPCHK(hipEventRecord(ev_[1], stream_));
    if (dec) HIPCHK(launch_rec_decode(du_.p, rec_pos_.p, total, c, stream_));
  }
  if (fused && spec_tail) {  // (then total == bound: no block stopped the span)
    out->next_pos = spec_next;  // (done and read with k_rec_check_out's verdict)
    out->first_voff = spec_voff[0];
    out->last_voff = spec_voff[1];
  } else {
    if (total) {
      HIPCHK(rb(&out->first_voff, rec_voff_.p, 8, stream_));
      HIPCHK(rb(&out->last_voff, rec_voff_.p + total - 1, 8, stream_));
    }
    if (dec) HIPCHK(launch_long_hash(du_.p, rec_pos_.p, c, stream_));
    // the next record's start: the chain successor of the last record
    HIPCHK(scalars_.reserve(8));
    HIPCHK(launch_next_pos(du_.p, rec_pos_.p, total, p0, mode, scalars_.p, stream_));
    HIPCHK(rb(&out->next_pos, scalars_.p, 8, stream_));
    if (timing) HIPCHK(hipEventRecord(ev_[2], stream_));
    HIPCHK(rb_sync(stream_));
  }
  if (after_stop_pending_ && after_stop_flag_) ++records_after_stop_;
  after_stop_pending_ = false;
  after_stop_flag_ = 0;
  if (timing) {
    float all = 0, dcd = 0;
    (void)hipEventElapsedTime(&all, ev_[0], ev_[1]);
    (void)hipEventElapsedTime(&dcd, ev_[1], ev_[2]);
    times.chain = all - infl_ms;
    times.decode = dcd;
    times.inflate = infl_ms;
    times.huff = huff_ms;
    times.lz77 = lz_ms;
    times.tables = tab_ms;
  }
  return kOk;
}

int Pipeline::alloc_columns(uint64_t total, uint64_t stream_bytes, Columns* cp, bool zero_long_n) {
  // SoA backing store: 8-byte columns first, then 4, 2, 1 (alignment)
  const uint64_t n = std::max<uint64_t>(total, 1);
  const uint64_t per = 8 * 2 + 4 * 7 + 2 * 3 + 1 * 2;
  if (cols_cap_ < n) {
    HIPCHK(cols_.reserve(n * per + 256));
    cols_cap_ = n;
  }
  HIPCHK(rec_voff_.reserve(n + 1));
  uint8_t* p = cols_.p;
  auto take = [&](uint64_t bytes) {
    uint8_t* r = p;
    p += (bytes + 15) & ~15ull;
    return r;
  };
  Columns& c = *cp;
  c.key = reinterpret_cast<int64_t*>(take(8 * n));
  c.rest_off = reinterpret_cast<uint64_t*>(take(8 * n));
  c.voff = rec_voff_.p;
  c.ref_id = reinterpret_cast<int32_t*>(take(4 * n));
  c.pos = reinterpret_cast<int32_t*>(take(4 * n));
  c.l_seq = reinterpret_cast<int32_t*>(take(4 * n));
  c.next_ref_id = reinterpret_cast<int32_t*>(take(4 * n));
  c.next_pos = reinterpret_cast<int32_t*>(take(4 * n));
  c.tlen = reinterpret_cast<int32_t*>(take(4 * n));
  c.rest_len = reinterpret_cast<uint32_t*>(take(4 * n));
  c.bin = reinterpret_cast<uint16_t*>(take(2 * n));
  c.n_cigar = reinterpret_cast<uint16_t*>(take(2 * n));
  c.flag = reinterpret_cast<uint16_t*>(take(2 * n));
  c.l_read_name = take(n);
  c.mapq = take(n);
  // deferred long-record keys: at most one per kLongHash stream bytes
  const uint64_t cap = std::min<uint64_t>(stream_bytes / kLongHash + 64, 0xffffffffull);
  HIPCHK(long_rec_.reserve(cap));
  HIPCHK(long_n_.reserve(1));
  if (zero_long_n) HIPCHK(hipMemsetAsync(long_n_.p, 0, 4, stream_));
  c.long_rec = long_rec_.p;
  c.long_n = long_n_.p;
  c.long_cap = (uint32_t)cap;
  return kOk;
}

int Pipeline::encoded_bytes(const SpanDev& s, uint64_t* bytes) {
  *bytes = 0;
  if (s.n == 0) return kOk;
  if (!s.col.rest_off) return fail(kErrState, "span was not decoded in reader mode");
  uint64_t first = 0, last_off = 0;
  uint32_t last_len = 0;
  HIPCHK(rb(&first, s.rec_pos, 8, stream_));
  HIPCHK(rb(&last_off, s.col.rest_off + (s.n - 1), 8, stream_));
  HIPCHK(rb(&last_len, s.col.rest_len + (s.n - 1), 4, stream_));
  HIPCHK(rb_sync(stream_));
  *bytes = last_off + last_len - first;
  return kOk;
}

int Pipeline::encode_writables(const SpanDev& s, uint64_t bytes, uint8_t* dst) {
  if (s.n == 0) return kOk;
  if (!s.col.ref_id) return fail(kErrState, "span was not decoded in reader mode");
  uint64_t first = 0;
  HIPCHK(rb(&first, s.rec_pos, 8, stream_));
  HIPCHK(rb_sync(stream_));
  const uint8_t* src = s.data ? s.data : du_.p;
  HIPCHK(launch_wr_encode(src, first, bytes, s.rec_pos, s.col.ref_id, s.col.bin, s.n, dst, stream_));
  return kOk;
}

int Pipeline::decode_writables(const uint8_t* buf, uint64_t len, const uint64_t* offs, uint64_t n, SpanDev* out) {
  *out = SpanDev();
  // 64 zero bytes after the values: the 8-byte field loads and Murmur's tail
  // loads may read past the last value
  HIPCHK(wbuf_.reserve(len + 64));
  HIPCHK(woffs_.reserve(n + 1));
  HIPCHK(wbad_.reserve(1));
  HIPCHK(rec_pos_.reserve(n + 1));
  if (len) HIPCHK(hipMemcpyAsync(wbuf_.p, buf, len, hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemsetAsync(wbuf_.p + len, 0, 64, stream_));
  if (n) HIPCHK(hipMemcpyAsync(woffs_.p, offs, n * 8, hipMemcpyHostToDevice, stream_));
  HIPCHK(hipMemsetAsync(wbad_.p, 0xff, sizeof(unsigned long long), stream_));
  Columns c{};
  int rc = alloc_columns(n, len, &c);
  if (rc != kOk) return rc;
  HIPCHK(launch_wr_decode(wbuf_.p, len, woffs_.p, n, c, rec_pos_.p, wbad_.p, stream_));
  HIPCHK(launch_long_hash(wbuf_.p, rec_pos_.p, c, stream_));
  unsigned long long bad = ~0ull;
  HIPCHK(rb(&bad, wbad_.p, sizeof bad, stream_));
  HIPCHK(rb_sync(stream_));
  out->n = n;
  if (bad != ~0ull) {
    out->n = bad >> 8;
    out->status = (int)(bad & 0xff);
    const std::string at = "value " + std::to_string(out->n);
    if (out->status == kErrFormat) out->error = "Invalid record length (" + at + ")";
    else if (out->status == kErrTrunc) out->error = "Premature EOF in serialized record (" + at + ")";
    else out->error = "value framing outside the buffer (" + at + ")";
  }
  out->p0 = 0;
  out->rec_pos = rec_pos_.p;
  out->rec_voff = rec_voff_.p;
  out->col = c;
  out->data = wbuf_.p;
  return kOk;
}

int Pipeline::splitting_entries(const SpanDev& span, uint32_t g, uint64_t o0, std::vector<uint64_t>* out) {
  out->clear();
  // global ordinals o0 .. o0+n-1; entries at ordinals k*g - 1
  const uint64_t m = (o0 + span.n) / g - o0 / g;
  if (m == 0) return kOk;
  DevBuf<uint64_t> ent(&streams_);
  HIPCHK(ent.reserve(m));
  HIPCHK(launch_sbi_emit(span.rec_voff, span.n, g, o0, ent.p, stream_));
  out->resize(m);
  HIPCHK(rb(out->data(), ent.p, m * 8, stream_));
  HIPCHK(rb_sync(stream_));
  return kOk;
}

int Pipeline::span_digest(const SpanDev& span, uint64_t out[4]) {
  out[0] = out[1] = out[2] = out[3] = 0;
  if (span.n == 0) return kOk;
  HIPCHK(scalars_.reserve(8));
  HIPCHK(hipMemsetAsync(scalars_.p + 2, 0, 32, stream_));
  HIPCHK(launch_digest(span.col.key, span.rec_voff, span.n, scalars_.p + 2, stream_));
  HIPCHK(rb(out, scalars_.p + 2, 32, stream_));
  HIPCHK(rb_sync(stream_));
  return kOk;
}

}  // namespace hbam
