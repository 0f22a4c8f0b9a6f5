// hbam_cursor.cpp -- SpanCursor: the drop-in batch iteration behind
// hbam_decode_span / BAMRecordReader.nextKeyValue (BAMRecordReader.java:
// 223-232), with the next batch and the next window in flight (hbam_host.h).
//
// Per window: BamFile::decode_step decodes it in the pipeline, k_export_records
// + k_pack_rests move its records (columns, record bytes, rests) into window slot
// (id % 2), positions rebased to the slot.  Per batch (records [k, k + m) of
// one window): three boundary reads (record k's start, the batch end, the
// read-ahead record's end) and the next voff, gathered by one small kernel on
// the meta stream, then the batch's columns (one batch-major block) and its
// rests (no fixed fields) go HBM -> page-locked host slot on the d2h stream.  Both are
// high-priority streams, on hardware queues of their own (hbam_pipeline.h).
// The batch handed out lives in one host slot while the next one fills the
// other.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "hbam_host.h"
#include "hbam_launch.h"
#include "hbam_mem.h"

namespace hadoop_bam {

using hbam::BlockInfo;
using hbam::ColLayout;
using hbam::kErrDevice;
using hbam::kErrNoMem;
using hbam::kErrState;
using hbam::kOk;

namespace {
// HBAM_CURSOR_TRACE: developer timing lines on stderr (ms since the last one)
bool cursor_trace() {
  static const bool t = getenv("HBAM_CURSOR_TRACE") != nullptr;
  return t;
}
void ctrace(const char* what, uint64_t a = 0) {
  if (!cursor_trace()) return;
  static auto last = std::chrono::steady_clock::now();
  const auto now = std::chrono::steady_clock::now();
  fprintf(stderr, "[cursor] +%.3f ms %s %llu\n", std::chrono::duration<double, std::milli>(now - last).count(), what,
          (unsigned long long)a);
  last = now;
}

hbam::Columns offset_columns(const hbam::Columns& c, uint64_t k) {
  hbam::Columns o = c;
  o.ref_id += k;
  o.pos += k;
  o.l_seq += k;
  o.next_ref_id += k;
  o.next_pos += k;
  o.tlen += k;
  o.l_read_name += k;
  o.mapq += k;
  o.bin += k;
  o.n_cigar += k;
  o.flag += k;
  o.key += k;
  o.voff += k;
  o.rest_off += k;
  o.rest_len += k;
  return o;
}

int hip_err(hipError_t e, const char* what, std::string* err) {
  if (e == hipSuccess) return kOk;
  *err = std::string(what) + ": " + hipGetErrorString(e);
  return kErrDevice;
}
#define CCHK(expr)                                      \
  do {                                                  \
    const int _rc = hip_err((expr), #expr, err);        \
    if (_rc != kOk) return _rc;                         \
  } while (0)
}  // namespace

SpanCursor::~SpanCursor() {
  join_prealloc();
  if (device_ < 0) return;
  (void)hipSetDevice(device_);
  (void)drain();
  (void)own_.sync();
  own_.n = 0;  // drained: the slot buffers release without waiting
  slot_owner_.n = 0;
  for (auto& w : win_) {
    w.cols.release();
    w.bytes.release();
    w.packed.release();
    w.rests.release();
    if (w.ready) (void)hipEventDestroy(w.ready);
  }
  for (auto& s : slot_) {
    if (s.mem) hbam::pinned_free(s.mem, s.cap);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (small_) (void)hipHostFree(small_);
  for (hipStream_t s : {d2h_, meta_})
    if (s) (void)hipStreamDestroy(s);
}

int SpanCursor::ensure_streams(hbam::Pipeline& p, std::string* err) {
  if (device_ == p.device() && own_.s[0] == p.stream()) return kOk;
  if (device_ >= 0) {  // another pipeline: drain everything of the old one
    (void)drain();
    (void)own_.sync();
  }
  CCHK(hipSetDevice(p.device()));
  if (device_ != p.device()) {
    if (d2h_) (void)hipStreamDestroy(d2h_);
    if (meta_) (void)hipStreamDestroy(meta_);
    CCHK(hbam::create_stream(&d2h_, hbam::StreamLevel::kHigh));  // own queues (hbam_pipeline.h)
    CCHK(hbam::create_stream(&meta_, hbam::StreamLevel::kHigh));
    if (!small_) CCHK(hipHostMalloc(reinterpret_cast<void**>(&small_), 64, hipHostMallocDefault));
    for (auto& w : win_)
      if (!w.ready) CCHK(hipEventCreateWithFlags(&w.ready, hipEventDisableTiming));
    for (auto& s : slot_)
      if (!s.done) CCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  device_ = p.device();
  own_.s[0] = p.stream();
  own_.s[1] = d2h_;
  own_.s[2] = meta_;
  own_.n = 3;
  slot_owner_.s[0] = p.stream();
  slot_owner_.n = 1;
  for (auto& w : win_) w.cols.owner = w.bytes.owner = w.packed.owner = w.rests.owner = &slot_owner_;
  return kOk;
}

int SpanCursor::drain() {
  for (auto& s : slot_) s.busy = false;
  if (device_ < 0) return kOk;
  const hipError_t a = hipStreamSynchronize(d2h_), b = hipStreamSynchronize(meta_);
  return a == hipSuccess && b == hipSuccess ? kOk : kErrDevice;
}

void SpanCursor::reset() {
  (void)drain();
  valid_ = false;
  last_bounded_ = false;
  last_m_ = 0;
  all_.n = 0;
  all_seg_.clear();
  nwin_ = front_ = k_ = 0;
}

uint64_t SpanCursor::block_end(const std::vector<BlockInfo>& B, uint64_t pos) const {
  // the non-empty block holding window position pos: file offset just past it
  uint64_t lo = 0, hi = B.size();
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (B[mid].ustart + B[mid].isize > pos) hi = mid; else lo = mid + 1;
  }
  if (lo >= B.size()) return B.empty() ? 0 : B.back().coff + B.back().csize;
  return B[lo].coff + B[lo].csize;
}

// Window sizes of a bounded split: the first batch cannot leave before the
// first window is copied and decoded, and nothing else overlaps that wait, so
// the windows ramp up from kRampFirst by kRampGrowth per window to the
// drop-in window, and the first batches cross PCIe while the larger windows
// decode.  HBAM_DROPIN_RAMP="<first MiB>,<growth>" (developer knob; "0": every
// window full size).
uint64_t SpanCursor::ramp_window(uint64_t full, uint64_t id) {
  struct Ramp {
    uint64_t first;
    double growth;
  };
  static const Ramp r = [] {
    Ramp v{32ull << 20, 2.0};
    if (const char* e = getenv("HBAM_DROPIN_RAMP")) {
      double mib = 0, g = 2.0;
      if (sscanf(e, "%lf,%lf", &mib, &g) >= 1) v = Ramp{(uint64_t)(mib * (1 << 20)), g > 1.0 ? g : 2.0};
    }
    return v;
  }();
  if (r.first == 0 || r.first >= full) return full;
  double w = (double)r.first;
  for (uint64_t k = 0; k < id && w < (double)full; ++k) w *= r.growth;
  return w < (double)full ? ((uint64_t)w + 0xffff) & ~0xffffull : full;
}

int SpanCursor::decode_window(BamFile& f, Carry from, bool cont, uint64_t m, Window* w, std::string* err) {
  // w's buffers are reused (reserve may hand a block back to the process
  // cache, dev_free does not wait for the device): no batch of the window
  // they hold may still be crossing PCIe.  next_batch re-decodes a window slot
  // only after its batches landed; this makes that explicit.
  for (const Slot& s : slot_)
    if (s.busy && s.win == w->id) CCHK(hipEventSynchronize(s.done));
  Step st;
  ctrace("decode_window start", nwin_);
  const uint64_t full = f.dropin_window_bytes();
  // ramped windows grow the staging buffer at every window: size it once for
  // the whole window up front, while nothing is in flight
  if (nwin_ == 0 && ramp_window(full, 0) < full) {
    const int r = f.pipe().reserve_stage(std::min<uint64_t>(full, f.file_size()));
    if (r != kOk) {
      *err = f.pipe().error();
      return r;
    }
  }
  int rc = f.decode_step(from, vend_, hbam::kReader, true, cont, &st, ramp_window(full, nwin_),
                         ramp_window(full, nwin_ + 1));
  ctrace("decode_step done", st.span.n);
  if (rc != kOk) {
    *err = f.error();
    return rc;
  }
  hbam::Pipeline& p = f.pipe();
  const SpanDev& s = st.span;
  w->id = nwin_;
  w->n = s.n;
  w->base_pos = s.p0;  // reader mode: the first record starts at p0
  w->nbytes = s.n ? s.next_pos - s.p0 : 0;
  w->next = st.next;
  w->ended = st.ended;
  w->status = st.status;
  w->error = st.error;
  w->blocks = std::make_shared<const std::vector<BlockInfo>>(p.blocks().begin(), p.blocks().end());
  w->pack_m = 0;
  if (s.n) {
    const ColLayout L(s.n, true);
    CCHK(w->cols.reserve(L.bytes));
    CCHK(w->bytes.reserve(w->nbytes + 16));
    w->col = L.at(w->cols.p, &w->rec_pos);
    if (m) {  // batch-major columns for batches of m records (the caller's batch size)
      const uint64_t nb = (s.n + m - 1) / m;
      CCHK(w->packed.reserve((nb - 1) * ColLayout(m, false).bytes + ColLayout(s.n - (nb - 1) * m, false).bytes));
      w->pack_m = m;
    }
    CCHK(hbam::launch_export_records(s.col, s.rec_pos, w->col, w->rec_pos, s.n, s.p0, w->nbytes,
                                     w->pack_m ? w->packed.p : nullptr, w->pack_m, p.stream()));
    // the record bytes (encode_writables of the last batch) and the rests alone (the batches)
    const uint8_t* u = s.data ? s.data : p.d_u();
    CCHK(hipMemcpyAsync(w->bytes.p, u + s.p0, w->nbytes, hipMemcpyDeviceToDevice, p.stream()));
    CCHK(w->rests.reserve(w->nbytes - 36 * s.n + 16));
    CCHK(hbam::launch_pack_rests(u, s.col.rest_off, s.col.rest_len, s.n, s.p0, w->rests.p, p.stream()));
  }
  CCHK(hipEventRecord(w->ready, p.stream()));
  ctrace("export queued");
  return kOk;
}

// First open of a split with batches of m records: both host slots are
// allocated on a helper thread while the first window decodes (mapping and
// pinning 2 x ~0.45 GB for 1 M-record batches took ~35 ms of the first
// batch).  The estimate is the columns plus 400 B of rests per record
// (150 bp reads: ~304); a bigger batch reallocates in issue() as before.
void SpanCursor::start_prealloc(uint64_t m, int device) {
  join_prealloc();
  const size_t est = ColLayout(m, false).bytes + 400 * m + 64;
  if (slot_[0].cap >= est && slot_[1].cap >= est) return;
  const int dev = device >= 0 ? device : device_;
  prealloc_ = std::thread([this, est, dev]() {
    if (hipSetDevice(dev) != hipSuccess) return;  // (the NUMA node of the allocation follows the device)
    for (auto& s : slot_) {
      if (s.cap >= est) continue;
      void* q = nullptr;
      size_t got = 0;
      if (hbam::pinned_alloc(&q, est + est / 8, &got) != hipSuccess) return;  // issue() tries again
      if (s.mem) hbam::pinned_free(s.mem, s.cap);
      s.mem = static_cast<uint8_t*>(q);
      s.cap = got;
    }
  });
}

void SpanCursor::join_prealloc() {
  if (prealloc_.joinable()) prealloc_.join();
}

// Rest bytes a bounded batch may hand out: below 2 GiB, the largest direct
// ByteBuffer (HBAM_MAX_BATCH_BYTES lowers it, for tests).
static uint64_t batch_data_cap() {
  const char* e = getenv("HBAM_MAX_BATCH_BYTES");
  const uint64_t hard = (1ull << 31) - 1024;
  const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
  return v && v < hard ? v : hard;
}

int SpanCursor::capped(const Window& w, uint64_t k, uint64_t m, uint64_t* out, std::string* err) {
  *out = m;
  const uint64_t cap = batch_data_cap();
  if (m <= 1 || w.nbytes - 36 * w.n <= cap) return kOk;  // the whole window fits: no reads
  // rests of records [k, e): (rec_pos[e] - rec_pos[k]) - 36 (e - k)
  auto rests = [&](uint64_t e, uint64_t* r) -> int {
    CCHK(hipStreamWaitEvent(meta_, w.ready, 0));
    const uint64_t* src[2] = {w.rec_pos + k, w.rec_pos + e};
    CCHK(hbam::launch_gather_u64(small_ + 6, src, 2, meta_));
    CCHK(hipStreamSynchronize(meta_));
    *r = (small_[7] - small_[6]) - 36 * (e - k);
    return kOk;
  };
  uint64_t r = 0;
  if (int rc = rests(k + m, &r)) return rc;
  if (r <= cap) return kOk;
  uint64_t lo = 1, hi = m;  // rests(k + lo) fits (one record always goes), rests(k + hi) does not
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (int rc = rests(k + mid, &r)) return rc;
    if (r <= cap) lo = mid; else hi = mid;
  }
  *out = lo;
  return kOk;
}

int SpanCursor::issue(const Window& w, uint64_t k, uint64_t m, Slot* s, std::string* err) {
  join_prealloc();
  // batch boundaries: record k's start, the batch end, the read-ahead
  // record's end (slot positions) and the next record's voff
  const uint64_t e = k + m;
  CCHK(hipStreamWaitEvent(meta_, w.ready, 0));
  // read by a kernel: a DMA copy would queue behind the other slot's batch
  const uint64_t* bounds[4] = {w.rec_pos + k, w.rec_pos + e, w.rec_pos + std::min(e + 1, w.n), w.col.voff + e};
  CCHK(hbam::launch_gather_u64(small_, bounds, e < w.n ? 4 : 3, meta_));
  CCHK(hipStreamSynchronize(meta_));
  s->win = w.id;
  s->k = k;
  s->m = m;
  s->start = small_[0];
  s->end = small_[1];
  s->ahead_end = e < w.n ? small_[2] : ~0ull;
  s->next_voff = e < w.n ? small_[3] : ~0ull;
  const ColLayout L(m, false);
  // the batch's rests: [start - 36 k, end - 36 e) of the window's packed rests
  const uint64_t rest_lo = s->start - 36 * k, rest_bytes = (s->end - s->start) - 36 * m;
  const size_t need = L.bytes + rest_bytes + 64;
  if (s->cap < need) {
    if (s->mem) hbam::pinned_free(s->mem, s->cap);
    s->mem = nullptr;
    s->cap = 0;
    void* q = nullptr;
    size_t got = 0;
    // headroom: the batches of a split differ a little in size
    if (hbam::pinned_alloc(&q, need + need / 8, &got) != hipSuccess) {
      *err = "page-locked host memory for the batch";
      return kErrNoMem;
    }
    s->mem = static_cast<uint8_t*>(q);
    s->cap = got;
  }
  const hbam::Columns src = offset_columns(w.col, k);
  uint8_t* h = s->mem;
  auto col = [&](int c, const void* from) {
    return hipMemcpyAsync(h + L.off[c], from, m * ColLayout::size_of(c), hipMemcpyDeviceToHost, d2h_);
  };
  CCHK(hipStreamWaitEvent(d2h_, w.ready, 0));
  // the batch-major copy of the columns when this batch is one of its blocks
  // (block k / pack_m holds min(pack_m, n - k) records)
  s->packed = w.pack_m && k % w.pack_m == 0 && m == std::min(w.pack_m, w.n - k);
  // rest_off stays on the device: the rests are back to back, so the host
  // takes it as the prefix sum of rest_len when the batch lands (next_batch);
  // 8 of a record's ~364 bytes on a link-bound loop
  if (s->packed) {
    const uint8_t* blk = w.packed.p + (k / w.pack_m) * ColLayout(w.pack_m, false).bytes;
    CCHK(hipMemcpyAsync(h, blk, L.off[ColLayout::kRestOff], hipMemcpyDeviceToHost, d2h_));
    CCHK(hipMemcpyAsync(h + L.off[ColLayout::kVoff], blk + L.off[ColLayout::kVoff], L.bytes - L.off[ColLayout::kVoff],
                        hipMemcpyDeviceToHost, d2h_));
  } else {
    CCHK(col(ColLayout::kKey, src.key));
    CCHK(col(ColLayout::kVoff, src.voff));
    CCHK(col(ColLayout::kRefId, src.ref_id));
    CCHK(col(ColLayout::kPos, src.pos));
    CCHK(col(ColLayout::kLSeq, src.l_seq));
    CCHK(col(ColLayout::kNextRefId, src.next_ref_id));
    CCHK(col(ColLayout::kNextPos, src.next_pos));
    CCHK(col(ColLayout::kTlen, src.tlen));
    CCHK(col(ColLayout::kRestLen, src.rest_len));
    CCHK(col(ColLayout::kBin, src.bin));
    CCHK(col(ColLayout::kNCigar, src.n_cigar));
    CCHK(col(ColLayout::kFlag, src.flag));
    CCHK(col(ColLayout::kLReadName, src.l_read_name));
    CCHK(col(ColLayout::kMapq, src.mapq));
  }
  if (rest_bytes) CCHK(hipMemcpyAsync(h + L.bytes, w.rests.p + rest_lo, rest_bytes, hipMemcpyDeviceToHost, d2h_));
  CCHK(hipEventRecord(s->done, d2h_));
  s->busy = true;
  ctrace("batch issued", k);
  return kOk;
}

int SpanCursor::next_batch(BamFile& f, uint64_t vstart, uint64_t vend, uint64_t max_records, BatchView* out,
                           uint64_t* next_voff, std::string* err) {
  *out = BatchView();
  hbam::Pipeline& p = f.pipe();
  int rc = ensure_streams(p, err);
  if (rc != kOk) return rc;
  if (max_records == 0) return next_batch_all(f, vstart, vend, out, next_voff, err);
  const bool cont = valid_ && last_bounded_ && vend == vend_ && vstart == next_voff_;
  if (!cont) {  // a seek to the split start (or anywhere in it)
    reset();
    vend_ = vend;
    start_prealloc(max_records);
    rc = decode_window(f, Carry{vstart >> 16, vstart & 0xffff}, false, max_records, &win_[0], err);
    if (rc != kOk) return rc;
    nwin_ = 1;
    valid_ = true;
  }
  last_bounded_ = true;
  last_m_ = 0;
  auto decode_next = [&](const Window& w) -> int {
    const int r = decode_window(f, w.next, true, max_records, &win_[nwin_ % 2], err);
    if (r != kOk) {
      valid_ = false;
      return r;
    }
    ++nwin_;
    return kOk;
  };
  // the front window with records left
  for (;;) {
    Window& W = win_[front_ % 2];
    if (k_ < W.n) break;
    if (W.ended) {  // the split is done (or ended at a failing record)
      *next_voff = W.status != kOk ? W.next.voff() : vend;
      next_voff_ = *next_voff;
      if (W.status != kOk) *err = W.error;
      return W.status;
    }
    if (nwin_ == front_ + 1 && (rc = decode_next(W)) != kOk) return rc;
    ++front_;
    k_ = 0;
  }
  Window& W = win_[front_ % 2];
  uint64_t m = 0;
  if ((rc = capped(W, k_, std::min(max_records, W.n - k_), &m, err)) != kOk) return rc;
  int s = -1;
  for (int j = 0; j < 2; ++j)
    if (slot_[j].busy && slot_[j].win == W.id && slot_[j].k == k_ && slot_[j].m == m) s = j;
  if (s < 0) {  // not prefetched (first batch, or the batch size changed)
    if ((rc = drain()) != kOk) return hip_err(hipErrorUnknown, "batch copy", err);
    s = cur_ == 0 ? 1 : 0;
    if ((rc = issue(W, k_, m, &slot_[s], err)) != kOk) return rc;
  }
  Slot& S = slot_[s];
  Slot& O = slot_[1 - s];
  // the next batch on the wire behind this one; the next window decoded
  // while this window's batches cross PCIe
  const bool in_window = k_ + m < W.n;
  uint64_t m2 = 0;
  if (in_window && ((rc = capped(W, k_ + m, std::min(max_records, W.n - k_ - m), &m2, err)) != kOk ||
                    (rc = issue(W, k_ + m, m2, &O, err)) != kOk))
    return rc;
  if (!W.ended && nwin_ == front_ + 1 && (rc = decode_next(W)) != kOk) return rc;
  const Window* N = nwin_ > front_ + 1 ? &win_[(front_ + 1) % 2] : nullptr;
  if (!in_window && N && N->n &&
      ((rc = capped(*N, 0, std::min(max_records, N->n), &m2, err)) != kOk || (rc = issue(*N, 0, m2, &O, err)) != kOk))
    return rc;
  // the read-ahead record past the window: the next window's first record
  uint64_t ahead = ~0ull;
  if (in_window) {
    ahead = block_end(*W.blocks, W.base_pos + S.ahead_end - 1);
  } else if (N && N->n) {
    uint64_t e1 = 0;
    CCHK(hipStreamWaitEvent(meta_, N->ready, 0));
    const uint64_t* src[1] = {N->rec_pos + 1};
    CCHK(hbam::launch_gather_u64(small_ + 4, src, 1, meta_));
    CCHK(hipStreamSynchronize(meta_));
    e1 = small_[4];
    ahead = block_end(*N->blocks, N->base_pos + e1 - 1);
  }
  ctrace("wait batch", k_);
  CCHK(hipEventSynchronize(S.done));
  ctrace("batch landed", k_);
  S.busy = false;
  // the batch: columns at ColLayout(m), the rests after them; rest_off in
  // the rests from the batch's first record, the prefix sum of rest_len
  // (issue() leaves it out of the copy)
  const ColLayout L(m, false);
  uint8_t* h = S.mem;
  const hbam::Columns c = L.at(h, nullptr);
  {
    uint64_t acc = 0;
    for (uint64_t i = 0; i < m; ++i) {
      c.rest_off[i] = acc;
      acc += c.rest_len[i];
    }
    if (acc != (S.end - S.start) - 36 * m) {
      valid_ = false;
      *err = "batch rest lengths do not add up to its record bytes";
      return kErrState;
    }
  }
  out->n = m;
  out->ref_id = c.ref_id;
  out->pos = c.pos;
  out->l_seq = c.l_seq;
  out->next_ref_id = c.next_ref_id;
  out->next_pos = c.next_pos;
  out->tlen = c.tlen;
  out->l_read_name = c.l_read_name;
  out->mapq = c.mapq;
  out->bin = c.bin;
  out->n_cigar = c.n_cigar;
  out->flag = c.flag;
  out->key = c.key;
  out->voff = c.voff;
  out->rest_off = c.rest_off;
  out->rest_len = c.rest_len;
  out->data = h + L.bytes;
  out->data_len = (S.end - S.start) - 36 * m;
  cur_ = s;
  last_win_ = W.id;
  last_k_ = k_;
  last_m_ = m;
  last_start_ = S.start;
  last_ahead_end_ = ahead;
  last_view_ = *out;
  last_blocks_ = W.blocks;
  last_base_pos_ = W.base_pos;
  k_ += m;
  int status = kOk;
  if (in_window) {
    *next_voff = S.next_voff;
  } else if (!W.ended) {
    *next_voff = W.next.voff();
  } else {
    status = W.status;
    if (status != kOk) *err = W.error;
    *next_voff = status != kOk ? W.next.voff() : vend;
  }
  next_voff_ = *next_voff;
  return status;
}

int SpanCursor::next_batch_all(BamFile& f, uint64_t vstart, uint64_t vend, BatchView* out, uint64_t* next_voff,
                               std::string* err) {
  reset();
  vend_ = vend;
  HostBatch& h = all_;
  h.n = 0;
  h.data_len = 0;
  h.window_pos.clear();
  all_seg_.clear();
  all_one_window_ = true;
  Carry c{vstart >> 16, vstart & 0xffff};
  bool cont = false;
  int status = kOk;
  int windows = 0;
  for (;;) {
    int rc = f.decode_step(c, vend, hbam::kReader, true, cont, &all_step_, f.dropin_window_bytes());
    if (rc != kOk) {
      *err = f.error();
      return rc;
    }
    ++windows;
    const SpanDev& s = all_step_.span;
    if (s.n) {
      all_seg_.emplace_back(h.n, std::make_shared<const std::vector<BlockInfo>>(f.pipe().blocks().begin(), f.pipe().blocks().end()));
      rc = fetch_span(f.pipe(), s, 0, s.n, &h, err);
      if (rc != kOk) return rc;
    }
    if (all_step_.ended) {
      status = all_step_.status;
      if (status != kOk) *err = all_step_.error;
      break;
    }
    c = all_step_.next;
    cont = true;
  }
  all_one_window_ = windows == 1;
  *out = BatchView::of(h);
  *next_voff = status != kOk ? all_step_.next.voff() : vend;
  next_voff_ = *next_voff;
  valid_ = true;
  last_bounded_ = false;
  last_view_ = *out;
  return status;
}

bool SpanCursor::last_batch_span(SpanDev* out) const {
  if (!valid_) return false;
  if (!last_bounded_) {
    if (!all_one_window_) return false;
    *out = all_step_.span;
    return true;
  }
  if (last_m_ == 0) return false;
  const Window& w = win_[last_win_ % 2];
  if (w.id != last_win_) return false;
  *out = SpanDev();
  out->n = last_m_;
  out->rec_pos = w.rec_pos + last_k_;
  out->rec_voff = w.col.voff + last_k_;
  out->col = offset_columns(w.col, last_k_);
  out->data = w.bytes.p;
  out->status = kOk;
  return true;
}

int SpanCursor::reader_position(uint64_t i, uint64_t* pos, std::string* err) const {
  // BAMRecordReader.getProgress (:209-219) reads in.position(): htsjdk's
  // iterator has already read the record after the one just returned (when
  // the split holds one), so the stream stands at the end of the block
  // holding that record's last byte.
  const BatchView& v = last_view_;
  if (!valid_ || i >= v.n) {
    *err = "no such record in the last batch";
    return kErrState;
  }
  auto last_byte_end = [&](uint64_t j) -> uint64_t {
    const uint64_t rel = v.rest_off[j] + v.rest_len[j] - 1;  // from data[0]
    // a bounded batch's data holds the rests alone: 36 B per record before j's end
    if (last_bounded_) return block_end(*last_blocks_, last_base_pos_ + last_start_ + rel + 36 * (j + 1));
    // whole-split batch: the segment (window) of record j
    size_t g = all_seg_.size() - 1;
    while (g > 0 && all_seg_[g].first > j) --g;
    return block_end(*all_seg_[g].second, all_.window_pos[g] + rel);
  };
  if (i + 1 < v.n) {
    *pos = last_byte_end(i + 1);
  } else if (last_bounded_ && last_ahead_end_ != ~0ull) {
    *pos = last_ahead_end_;
  } else {
    *pos = last_byte_end(i);  // the split holds no record after it
  }
  return kOk;
}

int SpanCursor::initial_position(uint64_t* pos, std::string* err) const {
  if (!valid_ || last_view_.n == 0) {
    *err = "no batch";
    return kErrState;
  }
  // record 0's own last byte (nothing has been read ahead yet)
  const uint64_t rel = last_view_.rest_off[0] + last_view_.rest_len[0] - 1;
  *pos = last_bounded_ ? block_end(*last_blocks_, last_base_pos_ + last_start_ + rel + 36)
                       : block_end(*all_seg_[0].second, all_.window_pos[0] + rel);
  return kOk;
}

}  // namespace hadoop_bam
