// hbam_feed.cpp -- HostFeed: threaded copies of pageable host bytes into
// page-locked bounce buffers, each piece DMA'd to HBM while the next fills
// (hbam_feed.h).
#include "hbam_feed.h"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "hbam_mem.h"

namespace hbam {

namespace {

// A fixed set of worker threads copying the parts of one piece at a time.
class CopyPool {
 public:
  explicit CopyPool(int threads) {
    for (int i = 1; i < threads; ++i) workers_.emplace_back([this] { work(); });
    parts_ = threads;
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  // dst[0, len) <- src[0, len), split over every thread of the pool (the
  // caller copies a part too); concurrent callers take turns
  void copy(uint8_t* dst, const uint8_t* src, size_t len) {
    std::lock_guard<std::mutex> turn(job_m_);
    if (workers_.empty() || len < (1u << 20)) {
      memcpy(dst, src, len);
      return;
    }
    Job j;
    {
      std::lock_guard<std::mutex> g(m_);
      j = Job{dst, src, len, ++gen_};
      job_ = j;
      left_ = parts_;
      ticket_.store(j.gen << 32);  // (job, next part)
    }
    cv_.notify_all();
    run_parts(j);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
  }

 private:
  struct Job {
    uint8_t* dst;
    const uint8_t* src;
    size_t len;
    uint64_t gen;
  };
  // parts of job j, claimed through the ticket; a thread still holding an
  // older job claims nothing of a newer one (the ticket carries the job)
  void run_parts(const Job& j) {
    const size_t per = ((j.len + parts_ - 1) / parts_ + 63) & ~size_t(63);  // 64 B-aligned parts
    for (;;) {
      uint64_t t = ticket_.load();
      if ((t >> 32) != j.gen || (int)(t & 0xffffffffu) >= parts_) return;
      if (!ticket_.compare_exchange_weak(t, t + 1)) continue;
      const size_t lo = (size_t)(t & 0xffffffffu) * per, hi = lo + per < j.len ? lo + per : j.len;
      if (lo < hi) memcpy(j.dst + lo, j.src + lo, hi - lo);
      std::lock_guard<std::mutex> g(m_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  void work() {
    uint64_t seen = 0;
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = job_;
      }
      run_parts(j);
    }
  }

  std::vector<std::thread> workers_;
  std::mutex job_m_;  // one job at a time
  std::mutex m_;
  std::condition_variable cv_, done_;
  bool stop_ = false;
  uint64_t gen_ = 0;
  int parts_ = 1;
  int left_ = 0;
  Job job_{};
  std::atomic<uint64_t> ticket_{0};
};

CopyPool& pool() {
  static CopyPool* p = new CopyPool(feed_threads());  // never destroyed: workers live as long as the process
  return *p;
}

}  // namespace

int feed_threads() {
  static const int n = [] {
    const char* e = getenv("HBAM_FEED_THREADS");
    int v = e ? atoi(e) : 8;
    return v < 1 ? 1 : v > 64 ? 64 : v;
  }();
  return n;
}

HostFeed::~HostFeed() {
  (void)drain();
  for (int i = 0; i < 2; ++i) {
    if (buf_[i]) pinned_free(buf_[i], cap_[i]);
    if (ev_[i]) (void)hipEventDestroy(ev_[i]);
  }
}

hipError_t HostFeed::drain() {
  for (int i = 0; i < 2; ++i)
    if (busy_[i]) {
      const hipError_t e = hipEventSynchronize(ev_[i]);
      if (e != hipSuccess) return e;
      busy_[i] = false;
    }
  return hipSuccess;
}

hipError_t HostFeed::copy(uint8_t* dst, const uint8_t* src, size_t len, hipStream_t s) {
  if (len == 0) return hipSuccess;
  if (len < kDirectBytes) return hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, s);
  hipError_t e;
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
  if (dev_ != dev) {  // events and buffers of another device: start afresh
    if ((e = drain()) != hipSuccess) return e;
    for (int i = 0; i < 2; ++i)
      if (ev_[i]) {
        (void)hipEventDestroy(ev_[i]);
        ev_[i] = nullptr;
      }
    dev_ = dev;
  }
  for (int i = 0; i < 2; ++i) {
    if (!buf_[i]) {
      void* p = nullptr;
      size_t got = 0;
      if ((e = pinned_alloc(&p, kPiece, &got)) != hipSuccess) return e;
      buf_[i] = static_cast<uint8_t*>(p);
      cap_[i] = got;
    }
    if (!ev_[i] && (e = hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming)) != hipSuccess) return e;
  }
  CopyPool& cp = pool();
  static const bool trace = getenv("HBAM_FEED_TRACE") != nullptr;  // developer timing lines on stderr
  using clk = std::chrono::steady_clock;
  for (size_t o = 0, k = 0; o < len; o += kPiece, ++k) {
    const int j = (int)(k & 1);
    const auto t0 = clk::now();
    if (busy_[j]) {  // this buffer's previous piece has crossed
      if ((e = hipEventSynchronize(ev_[j])) != hipSuccess) return e;
      busy_[j] = false;
    }
    const auto t1 = clk::now();
    const size_t n = len - o < kPiece ? len - o : kPiece;
    cp.copy(buf_[j], src + o, n);
    if (trace)
      fprintf(stderr, "[feed %p] piece %zu: wait %.3f ms, fill %.3f ms (%zu B)\n", (void*)this, k,
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(clk::now() - t1).count(), n);
    if ((e = hipMemcpyAsync(dst + o, buf_[j], n, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev_[j], s)) != hipSuccess) return e;
    busy_[j] = true;
  }
  return hipSuccess;
}

}  // namespace hbam
