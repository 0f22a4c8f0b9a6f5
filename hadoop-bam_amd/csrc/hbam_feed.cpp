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

#include <errno.h>
#include <sys/stat.h>
#include <unistd.h>

#include "hbam_device.h"
#include "hbam_mem.h"

namespace hbam {

int HostSource::read(uint8_t* dst, uint64_t off, uint64_t len, std::string* err) const {
  if (len == 0) return kOk;
  if (off > size || len > size - off) {
    *err = "read of [" + std::to_string(off) + ", " + std::to_string(off + len) + ") past the end of the " +
           std::to_string(size) + "-byte file";
    return kErrTrunc;
  }
  if (mem) {
    // a mapped path: a page past a shortened file's end would raise SIGBUS,
    // so the length is checked first (a truncation racing this copy can
    // still fault; HDFS block files and finished outputs are never cut)
    struct stat st;
    if (fd >= 0 && fstat(fd, &st) == 0 && (uint64_t)st.st_size < off + len) {
      *err = "file truncated: " + std::to_string((uint64_t)st.st_size) + " bytes now, " + std::to_string(size) +
             " when opened; read of [" + std::to_string(off) + ", " + std::to_string(off + len) + ")";
      return kErrTrunc;
    }
    memcpy(dst, mem + off, len);
    return kOk;
  }
  uint64_t done = 0;
  if (fd >= 0) {
    while (done < len) {
      const ssize_t r = pread(fd, dst + done, len - done, (off_t)(off + done));
      if (r < 0) {
        if (errno == EINTR) continue;
        *err = std::string("read error: ") + strerror(errno) + " at offset " + std::to_string(off + done);
        return kErrIO;
      }
      if (r == 0) break;
      done += (uint64_t)r;
    }
  } else if (read_fn) {
    std::unique_lock<std::mutex> g(mu, std::defer_lock);
    if (!concurrent) g.lock();
    while (done < len) {
      const int64_t r = read_fn(user, off + done, dst + done, len - done);
      if (r < 0) {
        *err = "read error (reader callback returned " + std::to_string(r) + ") at offset " + std::to_string(off + done);
        return kErrIO;
      }
      if (r == 0) break;
      done += (uint64_t)r;
    }
  } else {
    *err = "no host source";
    return kErrState;
  }
  if (done < len) {  // the file is shorter than when it was opened
    *err = "file truncated: " + std::to_string(done) + " of " + std::to_string(len) + " bytes at offset " +
           std::to_string(off) + " (the file was " + std::to_string(size) + " bytes when opened)";
    return kErrTrunc;
  }
  return kOk;
}

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
  void copy(uint8_t* dst, const uint8_t* src, size_t len) { (void)run(dst, src, nullptr, 0, len, nullptr); }
  // dst[0, len) <- bytes [off, off + len) of hs (status of the first failing part)
  int copy(uint8_t* dst, const HostSource& hs, uint64_t off, size_t len, std::string* err) {
    if (!hs.parallel()) return hs.read(dst, off, len, err);
    return run(dst, nullptr, &hs, off, len, err);
  }

 private:
  int run(uint8_t* dst, const uint8_t* src, const HostSource* hs, uint64_t off, size_t len, std::string* err) {
    std::lock_guard<std::mutex> turn(job_m_);
    if (workers_.empty() || len < (1u << 20)) {
      if (hs) return hs->read(dst, off, len, err);
      memcpy(dst, src, len);
      return kOk;
    }
    Job j;
    {
      std::lock_guard<std::mutex> g(m_);
      status_ = kOk;
      j = Job{dst, src, hs, off, len, ++gen_};
      job_ = j;
      left_ = parts_;
      ticket_.store(j.gen << 32);  // (job, next part)
    }
    cv_.notify_all();
    run_parts(j);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
    if (status_ != kOk && err) *err = status_msg_;
    return status_;
  }

  struct Job {
    uint8_t* dst;
    const uint8_t* src;
    const HostSource* hs;  // non-null: read [off, off + len) of it instead of src
    uint64_t off;
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
      int rc = kOk;
      std::string e;
      if (lo < hi) {
        if (j.hs) rc = j.hs->read(j.dst + lo, j.off + lo, hi - lo, &e);
        else memcpy(j.dst + lo, j.src + lo, hi - lo);
      }
      std::lock_guard<std::mutex> g(m_);
      if (rc != kOk && status_ == kOk) {
        status_ = rc;
        status_msg_ = e;
      }
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
  int status_ = kOk;  // the current job's first failing part
  std::string status_msg_;
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
  HostSource m;
  m.mem = src;
  m.size = len;
  std::string err;
  const int rc = copy(dst, m, 0, len, s, &err);
  return rc == kOk ? hipSuccess : rc == kErrDevice ? last_hip_ : hipErrorUnknown;
}

int HostFeed::copy(uint8_t* dst, const HostSource& src, uint64_t off, size_t len, hipStream_t s, std::string* err) {
  if (len == 0) return kOk;
  if (src.mem && src.fd < 0 && len < kDirectBytes) {  // (a mapped path: read() checks its length first)
    if (off > src.size || len > src.size - off) return src.read(nullptr, off, len, err);  // kErrTrunc
    last_hip_ = hipMemcpyAsync(dst, src.mem + off, len, hipMemcpyHostToDevice, s);
    if (last_hip_ != hipSuccess) *err = std::string("host->HBM copy: ") + hipGetErrorString(last_hip_);
    return last_hip_ == hipSuccess ? kOk : kErrDevice;
  }
  const int rc = pieces(dst, src, off, len, s, err);
  if (rc == kErrDevice && err->empty()) *err = std::string("host->HBM copy: ") + hipGetErrorString(last_hip_);
  return rc;
}

int HostFeed::pieces(uint8_t* dst, const HostSource& src, uint64_t off, size_t len, hipStream_t s, std::string* err) {
  hipError_t e;
#define FEEDCHK(x)                          \
  do {                                      \
    if ((e = (x)) != hipSuccess) {          \
      last_hip_ = e;                        \
      return kErrDevice;                    \
    }                                       \
  } while (0)
  int dev = 0;
  FEEDCHK(hipGetDevice(&dev));
  if (dev_ != dev) {  // events and buffers of another device: start afresh
    FEEDCHK(drain());
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
      FEEDCHK(pinned_alloc(&p, kPiece, &got));
      buf_[i] = static_cast<uint8_t*>(p);
      cap_[i] = got;
    }
    if (!ev_[i]) FEEDCHK(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming));
  }
  CopyPool& cp = pool();
  static const bool trace = getenv("HBAM_FEED_TRACE") != nullptr;  // developer timing lines on stderr
  using clk = std::chrono::steady_clock;
  for (size_t o = 0, k = 0; o < len; o += kPiece, ++k) {
    const int j = (int)(k & 1);
    const auto t0 = clk::now();
    if (busy_[j]) {  // this buffer's previous piece has crossed
      FEEDCHK(hipEventSynchronize(ev_[j]));
      busy_[j] = false;
    }
    const auto t1 = clk::now();
    const size_t n = len - o < kPiece ? len - o : kPiece;
    const int rc = cp.copy(buf_[j], src, off + o, n, err);
    if (rc != kOk) return rc;
    if (trace)
      fprintf(stderr, "[feed %p] piece %zu: wait %.3f ms, fill %.3f ms (%zu B)\n", (void*)this, k,
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(clk::now() - t1).count(), n);
    FEEDCHK(hipMemcpyAsync(dst + o, buf_[j], n, hipMemcpyHostToDevice, s));
    FEEDCHK(hipEventRecord(ev_[j], s));
    busy_[j] = true;
  }
  return kOk;
#undef FEEDCHK
}

}  // namespace hbam
