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

namespace hbam {

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
  // wait for every queued piece (before the caller frees dst or unmaps src)
  hipError_t drain();

  static constexpr size_t kPiece = 32ull << 20;
  static constexpr size_t kDirectBytes = 4ull << 20;

 private:
  uint8_t* buf_[2] = {nullptr, nullptr};
  size_t cap_[2] = {0, 0};
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool busy_[2] = {false, false};
  int dev_ = -1;
};

}  // namespace hbam
