// hbam_pipeline.h -- one HBM window of the BAM read hot path on one GPU.
//
// A Pipeline holds one window of a BGZF file: the compressed bytes [lo, hi)
// (copied from host memory or attached from a device-resident copy), its BGZF
// block table, the inflated stream of those blocks and the per-span record
// arrays.  A window that stops short of the end of the file is "open": a
// record that runs past its last block is not truncated, it is left for the
// next window (BamFile in hbam_host.h moves windows along a span and carries
// the next record's position across).  All compute runs in the gfx950
// kernels of hbam_kernels.hip; the host sizes buffers, launches and reads
// back counters.  There is no CPU fallback: any HIP failure is an error
// returned to the caller.
#pragma once
#include "hbam_feed.h"
#include "hbam_mem.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hbam_device.h"

namespace hbam {

// A device buffer.  `owner` = the streams that may have queued work on it
// (its Pipeline's): releasing or regrowing it waits for those streams only.
// A buffer without an owner waits for the whole device.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;  // elements
  const StreamSet* owner = nullptr;
  DevBuf() = default;
  explicit DevBuf(const StreamSet* o) : owner(o) {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void swap(DevBuf& o) {  // the contents; both keep their owner
    std::swap(p, o.p);
    std::swap(n, o.n);
  }
  hipError_t quiesce() const { return owner ? owner->sync() : hipDeviceSynchronize(); }
  void release() {
    if (p) {
      (void)quiesce();
      dev_free(p, n * sizeof(T));
    }
    p = nullptr;
    n = 0;
  }
  // grow, keeping the contents
  hipError_t grow(size_t count) {
    if (count <= n && p) return hipSuccess;
    const size_t c = count > 2 * n ? count : 2 * n;
    void* q = nullptr;
    size_t got = 0;
    hipError_t e = dev_alloc(&q, c * sizeof(T), &got);
    if (e != hipSuccess) return e;
    if (p) {
      if ((e = quiesce()) != hipSuccess) return e;
      // on the owner's stream: a plain hipMemcpy waits for the whole device
      if (owner && owner->n) {
        if ((e = hipMemcpyAsync(q, p, n * sizeof(T), hipMemcpyDeviceToDevice, owner->s[0])) != hipSuccess ||
            (e = hipStreamSynchronize(owner->s[0])) != hipSuccess)
          return e;
      } else if ((e = hipMemcpy(q, p, n * sizeof(T), hipMemcpyDeviceToDevice)) != hipSuccess) {
        return e;
      }
      dev_free(p, n * sizeof(T));
    }
    p = static_cast<T*>(q);
    n = got / sizeof(T);
    return hipSuccess;
  }
  // grow-only (contents not preserved)
  hipError_t reserve(size_t count) {
    if (count <= n && p) return hipSuccess;
    // half again the old size at least: a count that creeps up window by
    // window does not reallocate every time
    const size_t c = std::max<size_t>(count ? count : 1, p ? n + n / 2 : 0);
    release();
    void* q = nullptr;
    size_t got = 0;
    hipError_t e = dev_alloc(&q, c * sizeof(T), &got);
    if (e == hipSuccess) {
      p = static_cast<T*>(q);
      n = got / sizeof(T);
    }
    return e;
  }
};

// A page-locked host array of a trivially copyable T that kernels read or
// write in place (k_readback): the block table (54 K entries, 1.7 MB for C2)
// lands where the host reads it -- no zero fill on resize and no copy out of
// the read-back bounce buffer, ~0.11 ms of idle GPU per locate
// (profiles/r06/gaps.txt).
template <typename T>
class HostTable {
 public:
  HostTable() = default;
  HostTable(const HostTable&) = delete;
  HostTable& operator=(const HostTable&) = delete;
  ~HostTable() {
    if (p_) pinned_free(p_, bytes_);
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }
  const T& back() const { return p_[n_ - 1]; }
  void clear() { n_ = 0; }
  // keeps the first min(n, size()) elements, the others uninitialised; the
  // caller has waited for every kernel that reads or writes the array
  hipError_t resize(size_t n) {
    if (n > bytes_ / sizeof(T)) {
      void* q = nullptr;
      size_t got = 0;
      // at least 1 MiB: smaller page-locked blocks are not cached
      // (hbam_mem.cpp kMinCached), and hipHostFree waits for the device --
      // a drop-in context would pay it per window (ramped windows grow the
      // table several times per split)
      const size_t c = std::max(std::max(n, n_ + n_ / 2), (size_t(1) << 20) / sizeof(T));
      const hipError_t e = pinned_alloc(&q, c * sizeof(T), &got);
      if (e != hipSuccess) return e;
      if (n_) memcpy(q, p_, n_ * sizeof(T));
      if (p_) pinned_free(p_, bytes_);
      p_ = static_cast<T*>(q);
      bytes_ = got;
    }
    n_ = n;
    return hipSuccess;
  }

 private:
  T* p_ = nullptr;
  size_t n_ = 0, bytes_ = 0;
};

// Result of one span decode, resident on the device.
struct SpanDev {
  uint64_t n = 0;                 // records
  uint64_t p0 = 0, q_end = 0;     // window positions: span start, first position past the span
  uint64_t next_pos = 0;          // chain position after the last record (the next record's start)
  int status = kOk;               // status of the first failing record (records before it are valid)
  std::string error;
  uint64_t* rec_pos = nullptr;    // device
  uint64_t* rec_voff = nullptr;   // device
  uint64_t first_voff = 0, last_voff = 0;  // rec_voff[0], rec_voff[n - 1] (host; read back with the span)
  Columns col{};                  // device (reader mode + decode)
  const uint8_t* data = nullptr;  // device stream rec_pos / rest_off index (nullptr = the inflated stream)
};

struct StageTimes {  // milliseconds of the last decode (HIP events)
  float locate = 0, inflate = 0, huff = 0, lz77 = 0, chain = 0, decode = 0;
  float tables = 0;  // k_huff_tables (huff: k_inflate_huff only)
};

// Streams and hardware queues.  HIP maps streams onto GPU_MAX_HW_QUEUES
// hardware queues (default 4) per priority level, and a context drives seven
// streams: four decode streams, the staging copy, and the drop-in batches'
// D2H and small reads.  On a shared queue an event or stream wait queued
// behind a batch's D2H holds the decode kernels behind it (resident drop-in
// loop: 32 GB/s U on shared queues, 42-44 with 8 queues).  The decode
// streams take the normal level, the batch streams the high one and the
// staging copy the low one, so each gets its own queue at the default.
enum class StreamLevel { kNormal, kHigh, kLow };
hipError_t create_stream(hipStream_t* s, StreamLevel level);

// Record-level validation ([htsjdk] ValidationStringency, the
// hadoopbam.samheaderreader.validation-stringency property).
enum Stringency : int { kStrict = 0, kLenient = 1, kSilent = 2 };

class Pipeline {
 public:
  explicit Pipeline(int device);
  ~Pipeline();
  Pipeline(const Pipeline&) = delete;
  Pipeline& operator=(const Pipeline&) = delete;

  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  // every stream this pipeline queues work on (owner of its buffers and of
  // buffers its callers hand it: BamFile's resident copy, ABI temporaries)
  const StreamSet& streams() const { return streams_; }
  const std::string& error() const { return err_; }

  // Device -> host reads of the host logic, queued as k_readback launches on
  // stream s into a page-locked buffer (shader engines: a pageable D2H of the
  // block table waited ~13 ms behind a drop-in batch's D2H on another
  // stream).  The bytes land in dst when rb_sync(s) returns; rb_sync(s)
  // synchronizes s in any case.
  hipError_t rb(void* dst, const void* src, size_t bytes, hipStream_t s);
  hipError_t rb_sync(hipStream_t s);
  // dst (device) <- file bytes [off, off + len) of src through the copy
  // threads and bounce buffers (HostFeed), synchronously on the pipeline's
  // stream (a short read of src: kErrTrunc)
  int copy_from_host(uint8_t* dst, const HostSource& src, uint64_t off, uint64_t len);

  // Copy file bytes [base, base + len) into the window buffer.  at_eof: the
  // range ends at the end of the file (else the window is open).
  // When the window in place was loaded from the host too and holds a prefix
  // of the new range, that prefix moves device to device and only the rest
  // crosses PCIe; *host_bytes (optional) = the bytes copied from `data`.
  // (src: the file, read from offset base; data: its bytes [base, base + len) in memory)
  int load(const HostSource& src, uint64_t len, uint64_t base, bool at_eof, uint64_t* host_bytes = nullptr);
  int load(const uint8_t* data, uint64_t len, uint64_t base, bool at_eof, uint64_t* host_bytes = nullptr);
  // Start copying file bytes [lo, hi) of src into a staging buffer on the
  // copy stream; a later load() takes the part of its window inside [lo, hi)
  // from there (device-to-device) instead of the host, so a window's H2D
  // overlaps the previous window's decode.  src must outlive the copy.
  int stage(const HostSource& src, uint64_t lo, uint64_t hi);
  // the staging buffer sized for windows of up to `bytes` at once (growing it
  // later waits for the device)
  int reserve_stage(uint64_t bytes);
  // Use device-resident file bytes [base, base + len) (readable for kFilePad
  // bytes past len).
  int attach_device(const uint8_t* dptr, uint64_t len, uint64_t base, bool at_eof);
  // Copy the same-size window bytes into the resident buffer again, timed with
  // HIP events (PCIe-inclusive measurements); pinned: from a page-locked copy.
  int reload(const uint8_t* data, uint64_t len, bool pinned, float* ms);
  // hipMemcpy device-to-device bandwidth (read + write bytes per second / 1e9)
  int d2d_bandwidth(uint64_t bytes, int iters, float* gbps);
  uint64_t file_len() const { return flen_; }
  uint64_t base() const { return base_; }
  bool at_eof() const { return at_eof_; }
  const uint8_t* d_file() const { return dfile_; }

  // BGZF block discovery over the window.  An open window keeps only the
  // blocks that end inside it.  free_start: the window may begin inside a
  // block (split-guess windows); the block chain starts at the first header
  // candidate whose BSIZE chain runs to the window end.
  int locate(bool free_start = false);
  const HostTable<BlockInfo>& blocks() const { return hblocks_; }
  uint64_t total_u() const { return total_u_; }
  const BlockInfo* d_blocks() const { return dblocks_.p; }
  // file offset just past the last located block (where the next window starts)
  uint64_t window_end() const { return window_end_; }

  // Inflate blocks [b0, b1) into the contiguous inflated stream.  check =
  // false leaves the work queued (no DEFLATE error check, no host wait).
  // join: the last chunk's phase B runs on stream() itself (the caller's next
  // work needs it); else on the phase-B stream, beside what is queued next.
  int inflate(uint32_t b0, uint32_t b1, bool force = false, bool check = true, bool join = true);

  // End-to-end pass from host memory: the file (same length as the loaded
  // one) is copied to HBM in pieces on a copy stream while the BGZF blocks of
  // every piece that has landed are located and inflated, then the record
  // chain + decode run over the whole file (first record at stream position
  // first_pos).  data should be page-locked for the copies to overlap.
  // *ms = first copy to last decode (HIP events).
  int run_streamed(const uint8_t* data, uint64_t len, uint64_t piece_bytes, uint64_t first_pos, SpanDev* out,
                   float* ms);
  const uint8_t* d_u() const { return du_.p; }

  // Record chain over the span [vstart, vend) under reader or indexer rules;
  // decode=true also fills the SoA columns + keys (reader mode only).  In an
  // open window the span also ends at the first record that does not end
  // inside the window (out->next_pos = its start).
  int decode_span(uint64_t vstart, uint64_t vend, ChainMode mode, bool decode, SpanDev* out);
  // Same, from a window position (index mode: a carried position may lie
  // past the first block).
  int decode_span_pos(uint64_t p0, uint64_t vend, ChainMode mode, bool decode, SpanDev* out);

  // Header bytes: inflate the first blocks until `need` stream bytes exist.
  int read_stream(uint64_t pos, uint64_t len, std::vector<uint8_t>* out);

  // SAMRecordWritable.write (SAMRecordWritable.java:55-64) of every record of
  // a decoded reader span, back to back: *bytes = size of the encodings;
  // encode_writables writes them to dst (device; room for bytes rounded up
  // to 16).  Record i's encoding starts at rec_pos[i] - rec_pos[0].
  int encoded_bytes(const SpanDev& span, uint64_t* bytes);
  int encode_writables(const SpanDev& span, uint64_t bytes, uint8_t* dst);
  // SAMRecordWritable.readFields (SAMRecordWritable.java:65-68) of n values
  // framed by offs in host memory (value i = buf[offs[i], offs[i+1]), the
  // last ends at len): SoA columns + keys; out->n stops at the first bad value.
  int decode_writables(const uint8_t* buf, uint64_t len, const uint64_t* offs, uint64_t n, SpanDev* out);

  // .splitting-bai entries of a span whose first record has global ordinal
  // `ordinal0` (SplittingBAMIndexer.java:273-277: ordinals k*g - 1)
  int splitting_entries(const SpanDev& span, uint32_t granularity, uint64_t ordinal0, std::vector<uint64_t>* out);
  // digests of a decoded span (bench / test checks): key xor, voff sum and
  // the order-sensitive key / voff digests (k_digest)
  int span_digest(const SpanDev& span, uint64_t out[4]);

  // host helpers on the block table
  int64_t pos_of_voff(uint64_t voff) const;
  uint64_t voff_of(uint64_t pos) const;
  uint64_t q_end_of(uint64_t vend) const;
  uint32_t block_containing(uint64_t pos) const;  // non-empty block with ustart <= pos < end, or nblocks

  void set_n_ref(int32_t n) { n_ref_ = n; }
  int32_t n_ref() const { return n_ref_; }
  void set_stringency(int s) { stringency_ = s; }
  // reference lengths for the STRICT alignment-start checks (empty = none)
  int set_ref_lengths(const std::vector<int32_t>& lens);

  uint64_t link_fallbacks() const { return link_fallbacks_; }
  uint64_t link_rewalks() const { return link_rewalks_; }
  uint64_t record_fallbacks() const { return record_fallbacks_; }
  uint64_t records_after_stop() const { return records_after_stop_; }
  uint64_t inflate_launches() const { return inflate_launches_; }
  // LZ77 tokens phase A wrote for the window's blocks in its last inflate
  // (the sum of HuffOut::ntok; a synchronous read, for measurements)
  int inflate_tokens(uint64_t* n);
  StageTimes times;
  bool timing = false;  // record per-stage HIP event times

 private:
  int fail(int code, const std::string& msg);
  // BGZF blocks of [lo, hi) appended at index nprev with ustart from ubase,
  // on stream s (synchronized).  partial: a block cut by hi is left out and
  // *tail = its start (hi when none).
  int locate_range(uint64_t lo, uint64_t hi, bool partial, bool free_start, uint32_t nprev, uint64_t ubase,
                   hipStream_t s, uint32_t* nnew, uint64_t* tail);
  int finish_blocks();  // total_u_, dead positions, pads, per-block state after locate
  // the first failing block of [b0, b1)'s inflate, read back into
  // infl_first_ at the next rb_sync; inflate_verdict: its error, if any
  hipError_t queue_inflate_check(uint32_t b0, uint32_t b1);
  int inflate_verdict(uint32_t b0, uint32_t b1);
  uint32_t infl_first_ = 0xffffffffu;
  bool inflate_queued_ = false;  // the last inflate() queued any chunk
  // SoA store for n records (voff = rec_voff_) + the deferred long-key list
  int alloc_columns(uint64_t n, uint64_t stream_bytes, Columns* c, bool zero_long_n = true);
  int hip_check(hipError_t e, const char* what);

  template <typename... B>
  void own(B&... b) {
    ((b.owner = &streams_), ...);
  }

  int device_ = 0;
  StreamSet streams_;
  hipStream_t stream_ = nullptr;
  hipStream_t stream_copy_ = nullptr;  // run_streamed: host->HBM pieces
  hipStream_t stream_stage_ = nullptr;  // stage(): the next window's bytes (not in streams_)
  StreamSet stage_owner_;              // stage_'s owner: stream_stage_ + stream_
  std::vector<hipEvent_t> copy_ev_;
  std::string err_;

  uint8_t* dfile_ = nullptr;
  DevBuf<uint8_t> own_file_;  // window bytes copied from the host (+ kFilePad zeros)
  DevBuf<uint8_t> own_spare_;  // the other buffer of the pair (a window's kept prefix moves across)
  DevBuf<uint8_t> stage_;      // stage(): file bytes [stage_lo_, stage_hi_) in flight / landed
  uint64_t stage_lo_ = 0, stage_hi_ = 0;
  std::thread stage_thr_;      // issues the staged copy (pageable copies block their caller)
  HostFeed feed_load_, feed_stage_;  // host -> HBM copies of load() and of the stage thread
  int stage_rc_ = 0;           // the staged copy's status (kOk = 0) and message
  std::string stage_msg_;
  int stage_wait();            // the staged copy done (its error, if any)
  // load() of file bytes [base, base + len) read from src at src_off + (x - base)
  int load_from(const HostSource& src, uint64_t src_off, uint64_t len, uint64_t base, bool at_eof,
                uint64_t* host_bytes);
  uint64_t flen_ = 0, base_ = 0;
  bool at_eof_ = true;
  uint64_t window_end_ = 0;

  DevBuf<BlockInfo> dblocks_;
  HostTable<BlockInfo> hblocks_;  // read back in place (k_readback)
  HostTable<uint64_t> hdead_;      // dead positions, copied to dead_ by k_readback
  uint64_t total_u_ = 0;
  uint32_t ndead_ = 0;
  // empty blocks among hblocks_ (counted by the verify kernel), or unknown
  static constexpr uint32_t kEmptyUnknown = 0xffffffffu;
  uint32_t empty_blocks_ = kEmptyUnknown;
  int32_t n_ref_ = 0;
  int stringency_ = kStrict;
  DevBuf<int32_t> ref_len_;
  uint32_t n_ref_len_ = 0;
  uint64_t link_fallbacks_ = 0;
  uint64_t link_rewalks_ = 0;      // re-walk rounds of the parallel link
  uint64_t record_fallbacks_ = 0;  // spans whose lists overflowed: records counted and emitted by walks
  uint64_t records_after_stop_ = 0;  // spans that stopped early with records listed in later blocks (dropped)
  uint32_t after_stop_flag_ = 0;     // (read back with a span's last readback)
  bool after_stop_pending_ = false;
  uint64_t inflate_launches_ = 0;  // phase A/B launch pairs so far

  DevBuf<uint8_t> du_;
  std::vector<uint8_t> inflated_;  // per block flag
  DevBuf<uint32_t> tokens_[2];  // LZ77 token streams, by chunk parity (overlapped inflate)
  DevBuf<HuffOut> hout_;
  DevBuf<uint8_t> tables_[2];     // phase-A prebuilt table images (per chunk, by chunk parity)
  hipStream_t stream_b_ = nullptr;  // inflate phase B (overlaps phase A of the next chunk)
  hipStream_t stream_t_ = nullptr;  // round-0 table build of chunk j beside phase A of chunk j-1
  hipEvent_t tab_ev_[2];            // tables of the chunk of that parity built
  hipEvent_t hdone_ev_[2];          // phase A of the chunk of that parity done (tables free)
  hipEvent_t sync_ev_[4];           // [0,1] phase A done, [2,3] phase B done, per token buffer
  DevBuf<HuffTableInfo> tinfo_[2];

  // span scratch
  DevBuf<uint64_t> g_, x_, x2_, entry_, base_arr_, summary_, dead_;
  DevBuf<uint64_t> cand_, sorted_, isz_, ust_;  // locate scratch
  DevBuf<uint32_t> cnt_, flags_;
  DevBuf<int32_t> errv_;
  DevBuf<unsigned long long> need_;
  DevBuf<uint64_t> rec_pos_, rec_voff_;
  DevBuf<uint64_t> rcand_, force_;  // chain v2
  DevBuf<uint32_t> wcnt_, counters_;
  DevBuf<uint16_t> list_;
  DevBuf<uint32_t> fuse_;  // k_rec_check_out: [0..1] early-stop key (u64), [2] first failing block, [3] last block with records + 1
  DevBuf<uint8_t> scan_tmp_;
  DevBuf<uint8_t> cols_;  // SoA backing store
  uint64_t cols_cap_ = 0;
  DevBuf<uint64_t> long_rec_;            // records whose key k_long_hash computes
  DevBuf<uint32_t> long_n_;
  DevBuf<uint8_t> wbuf_;                 // readFields: serialized values
  DevBuf<uint64_t> woffs_;               // readFields: value framing
  DevBuf<unsigned long long> wbad_;      // readFields: first bad value
  DevBuf<uint64_t> scalars_;             // next_pos / digests read back by the host

  hipEvent_t ev_[8];
  std::vector<hipEvent_t> tev_;     // timing events of overlapped inflate chunks

  // read-back queue (rb / rb_sync)
  struct RbItem {
    void* dst;
    size_t off, bytes;
  };
  uint8_t* rb_buf_ = nullptr;
  size_t rb_cap_ = 0, rb_used_ = 0;
  hipStream_t rb_stream_ = nullptr;
  std::vector<RbItem> rb_items_;
};

}  // namespace hbam
