// hbam_feed.h -- host -> HBM copies of pageable bytes (a mapped BAM file) at
// the link rate.
//
// A pageable hipMemcpy pins each host page as it goes: from a fresh mapping
// of a /dev/shm C2 file it moves 11.7 GB/s (56 GB/s only for pages the
// runtime has seen before), and neither registering the mapping first
// (hipHostRegister, 1-16 threads: ~10 GB/s all in) nor pageable copies from
// several threads do better.  Worker threads that memcpy the mapping into
// page-locked bounce buffers take the page faults in parallel instead, and
// each filled piece crosses PCIe by DMA while the next one fills: 53 GB/s at
// 8 threads (scripts/h2d_map_probe.hip, the same box).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <string>

namespace hbam {

// Where a file's host bytes come from, the way BAMRecordReader reads through
// WrapSeekable (util/WrapSeekable.java:56-87): memory (an in-memory copy, or
// hbam_open's read-only mapping of the path, with fd set: each read first
// checks the file's length, so a file truncated under an open ctx fails with
// HBAM_E_TRUNC instead of a SIGBUS), a file descriptor read with pread (fd
// without mem), or a positioned-read callback (hbam_open_reader: a Hadoop
// FSDataInputStream, PositionedReadable.read(position, buf, off, len),
// through JNI).  The mapping stays: memcpy from it by the feed threads moved
// C3 at 108 GB/s U, pread into the bounce buffers at 47 (r04d).
struct HostSource {
  typedef int64_t (*ReadFn)(void* user, uint64_t offset, void* dst, uint64_t len);
  const uint8_t* mem = nullptr;
  int fd = -1;
  ReadFn read_fn = nullptr;
  void* user = nullptr;
  uint64_t size = 0;
  bool concurrent = false;  // read_fn may run on several threads at once (hbam_opts.parallel_reads)
  bool valid() const { return mem || fd >= 0 || read_fn; }
  // pieces of one copy may be read by several threads at once (memory, pread,
  // a concurrent callback); another callback is called by one thread at a time (mu)
  bool parallel() const { return read_fn == nullptr || concurrent; }
  // dst[0, len) <- file bytes [off, off + len): kOk, kErrTrunc (the file ends
  // before off + len) or kErrIO (a read error), with *err set
  int read(uint8_t* dst, uint64_t off, uint64_t len, std::string* err) const;
  mutable std::mutex mu;
};

// Copy threads of the process (the caller + workers): HBAM_FEED_THREADS, else
// 8.  Jobs of concurrent contexts take turns.
int feed_threads();

// One context's bounce buffers.  Not thread-safe: one copy() at a time.
class HostFeed {
 public:
  HostFeed() = default;
  ~HostFeed();
  HostFeed(const HostFeed&) = delete;
  HostFeed& operator=(const HostFeed&) = delete;
  // dst (device) <- src (host, any memory) [len): pieces filled by the copy
  // threads and queued on s; returns when the last piece is queued (its DMA
  // may still run: order later work after it on s, or synchronize s).
  // Copies below kDirectBytes go straight through hipMemcpyAsync.
  hipError_t copy(uint8_t* dst, const uint8_t* src, size_t len, hipStream_t s);
  // dst (device) <- file bytes [off, off + len) of src, the same way (a
  // source that is not memory always goes through the bounce buffers).
  // Returns kOk, kErrTrunc / kErrIO (src's read failed; *err says why) or
  // kErrDevice.
  int copy(uint8_t* dst, const HostSource& src, uint64_t off, size_t len, hipStream_t s, std::string* err);
  // wait for every queued piece (before the caller frees dst or unmaps src)
  hipError_t drain();

  static constexpr size_t kPiece = 32ull << 20;
  static constexpr size_t kDirectBytes = 4ull << 20;

 private:
  int pieces(uint8_t* dst, const HostSource& src, uint64_t off, size_t len, hipStream_t s, std::string* err);
  hipError_t last_hip_ = hipSuccess;
  uint8_t* buf_[2] = {nullptr, nullptr};
  size_t cap_[2] = {0, 0};
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool busy_[2] = {false, false};
  int dev_ = -1;
};

}  // namespace hbam
