// hbam_mem.cpp -- the block caches of hbam_mem.h.
#include "hbam_mem.h"

#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdlib>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <string>
#include <map>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

namespace hbam {
namespace {

// Every device block is cached, however small: hipFree waits for the whole
// device, so freeing even a 40 KB candidate list behind a drop-in batch's
// D2H held a window's locate for 13 ms.  Page-locked blocks below
// kMinCached are not worth keeping.  The caps bound what a process keeps
// after its splits close.
constexpr size_t kMinCached = 1ull << 20;
constexpr size_t kDevCap = 32ull << 30;     // of 288 GB HBM per MI355X
// Blocks below kMinCached have a cache of their own: once closed contexts'
// window buffers fill kDevCap, a small block freed by a running decode would
// otherwise go to hipFree (the drop-in loop after the bench's pinned-host leg
// ran at 23 GB/s U instead of 39).
constexpr size_t kDevSmallCap = 256ull << 20;
constexpr size_t kPinnedCap = 8ull << 30;

struct Cache {
  std::mutex mu;
  std::multimap<size_t, std::pair<void*, int>> blocks;  // size -> (pointer, device)
  size_t total = 0;

  // smallest cached block in [bytes, 2 * bytes] on `dev`
  void* take(size_t bytes, int dev, size_t* got) {
    std::lock_guard<std::mutex> lk(mu);
    for (auto it = blocks.lower_bound(bytes); it != blocks.end() && it->first <= 2 * bytes; ++it) {
      if (it->second.second != dev) continue;
      void* p = it->second.first;
      *got = it->first;
      total -= it->first;
      blocks.erase(it);
      return p;
    }
    return nullptr;
  }
  // empties the cache into `out` (freed by the caller, outside the lock)
  size_t drain(std::multimap<size_t, std::pair<void*, int>>* out) {
    std::lock_guard<std::mutex> lk(mu);
    out->swap(blocks);
    const size_t t = total;
    total = 0;
    return t;
  }
  bool put(void* p, size_t bytes, int dev, size_t cap) {
    std::lock_guard<std::mutex> lk(mu);
    if (total + bytes > cap) return false;
    blocks.emplace(bytes, std::make_pair(p, dev));
    total += bytes;
    return true;
  }
};

// never destroyed: blocks cached at exit go with the process (freeing them
// from a static destructor could run after the HIP runtime is torn down)
Cache& dev_cache() {
  static Cache* c = new Cache();
  return *c;
}
Cache& dev_small_cache() {
  static Cache* c = new Cache();
  return *c;
}
Cache& pinned_cache() {
  static Cache* c = new Cache();
  return *c;
}

int current_device() {
  int d = 0;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

}  // namespace

hipError_t dev_alloc(void** p, size_t bytes, size_t* got) {
  if (bytes == 0) bytes = 1;
  const int dev = current_device();
  if (void* q = (bytes < kMinCached ? dev_small_cache() : dev_cache()).take(bytes, dev, got)) {
    *p = q;
    return hipSuccess;
  }
  *got = bytes;
  return hipMalloc(p, bytes);
}

// the device a block lives on (the caller's current device may differ)
int device_of(void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) return -1;
  return a.device;
}

void dev_free(void* p, size_t bytes) {
  if (!p) return;
  const int dev = device_of(p);
  if (dev < 0) {
    (void)hipFree(p);
    return;
  }
  // the owner has drained its streams (DevBuf::release): no device-wide wait
  const bool kept = bytes < kMinCached ? dev_small_cache().put(p, bytes, dev, kDevSmallCap)
                                       : dev_cache().put(p, bytes, dev, kDevCap);
  if (!kept) (void)hipFree(p);
}

namespace {
// Large page-locked blocks are not hipHostMalloc'ed: that zero-fills every
// page on one thread (~96 ms per GiB on the MI355X box, scripts/pin_probe.py).
// They are mapped (2 MiB aligned, huge pages advised), first-touched on
// several threads, then registered (hipHostRegister: ~3 ms per GiB).
constexpr size_t kRegisterMin = 16ull << 20;
constexpr size_t kHuge = 2ull << 20;

std::mutex& reg_mu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
std::set<void*>& registered() {  // blocks from the map + register path
  static std::set<void*>* s = new std::set<void*>();
  return *s;
}

// The NUMA node of the current device (-1: unknown).  A host has several
// (the MI355X box: 2 sockets, its GPU on node 1), and a page-locked buffer
// first-touched by threads on the other socket crosses the socket link on
// every DMA: the drop-in batches' D2H ran at ~30 GB/s instead of 56 when the
// batch slots landed there.
int device_numa_node() {
  static std::mutex mu;
  static std::map<int, int> known;
  const int dev = current_device();
  if (dev < 0) return -1;
  std::lock_guard<std::mutex> lk(mu);
  auto it = known.find(dev);
  if (it != known.end()) return it->second;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) == hipSuccess) {
    for (char* c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    if (FILE* f = fopen(path.c_str(), "r")) {
      if (fscanf(f, "%d", &node) != 1) node = -1;
      fclose(f);
    }
  }
  known[dev] = node;
  return node;
}

void* map_and_touch(size_t bytes) {
  void* q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (q == MAP_FAILED) return nullptr;
  (void)madvise(q, bytes, MADV_HUGEPAGE);
  // pages on the device's node whichever CPUs touch them (preferred: another
  // node when that one is full)
  const int node = device_numa_node();
  if (node >= 0 && node < 64) {
    const unsigned long mask = 1ul << node;
    (void)syscall(SYS_mbind, q, bytes, 1 /* MPOL_PREFERRED */, &mask, 64ul, 0u);
  }
  const size_t nt = std::min<size_t>(8, std::max<size_t>(1, bytes / (32ull << 20)));
  const size_t per = (bytes / nt + kHuge - 1) & ~(kHuge - 1);
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([q, bytes, per, t]() {
      volatile uint8_t* b = static_cast<uint8_t*>(q);
      for (size_t o = t * per; o < std::min(bytes, (t + 1) * per); o += 4096) b[o] = 0;
    });
  for (auto& x : th) x.join();
  return q;
}

}  // namespace

hipError_t pinned_alloc(void** p, size_t bytes, size_t* got) {
  if (bytes == 0) bytes = 1;
  if (bytes >= kMinCached) {
    if (void* q = pinned_cache().take(bytes, 0, got)) {
      *p = q;
      return hipSuccess;
    }
  }
  if (bytes >= kRegisterMin) {
    const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
    void* q = map_and_touch(len);
    if (q) {
      const hipError_t e = hipHostRegister(q, len, hipHostRegisterDefault);
      if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(reg_mu());
        registered().insert(q);
        *p = q;
        *got = len;
        return hipSuccess;
      }
      munmap(q, len);
    }
  }
  *got = bytes;
  return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

namespace {
void pinned_release(void* p, size_t bytes) {
  bool reg = false;
  {
    std::lock_guard<std::mutex> lk(reg_mu());
    reg = registered().erase(p) != 0;
  }
  if (reg) {
    (void)hipHostUnregister(p);
    munmap(p, bytes);
  } else {
    (void)hipHostFree(p);
  }
}
}  // namespace

void pinned_free(void* p, size_t bytes) {
  if (!p) return;
  // every copy into a batch buffer is waited for by its owner (fetch_span,
  // the batch prefetch): no device-wide wait here
  if (bytes >= kMinCached && pinned_cache().put(p, bytes, 0, kPinnedCap)) return;
  pinned_release(p, bytes);
}

size_t release_cached() {
  std::multimap<size_t, std::pair<void*, int>> d, h;
  size_t n = dev_cache().drain(&d) + pinned_cache().drain(&h);
  {
    std::multimap<size_t, std::pair<void*, int>> small;
    n += dev_small_cache().drain(&small);
    d.insert(small.begin(), small.end());
  }
  const int cur = current_device();
  for (auto& b : d) {
    (void)hipSetDevice(b.second.second);
    (void)hipFree(b.second.first);
  }
  if (cur >= 0) (void)hipSetDevice(cur);
  for (auto& b : h) pinned_release(b.second.first, b.first);
  return n;
}

}  // namespace hbam
