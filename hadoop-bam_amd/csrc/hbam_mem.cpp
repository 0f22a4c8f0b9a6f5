// hbam_mem.cpp -- the block caches of hbam_mem.h.
#include "hbam_mem.h"

#include <map>
#include <mutex>

namespace hbam {
namespace {

// Blocks below kMinCached bytes are not worth caching (hipMalloc is cheap
// for them); the caps bound what a process keeps after its splits close.
constexpr size_t kMinCached = 1ull << 20;
constexpr size_t kDevCap = 32ull << 30;     // of 288 GB HBM per MI355X
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
  if (bytes >= kMinCached) {
    if (void* q = dev_cache().take(bytes, dev, got)) {
      *p = q;
      return hipSuccess;
    }
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
  const int dev = bytes >= kMinCached ? device_of(p) : -1;
  if (dev < 0) {
    (void)hipFree(p);
    return;
  }
  // the owner has drained its streams (DevBuf::release): no device-wide wait
  if (!dev_cache().put(p, bytes, dev, kDevCap)) (void)hipFree(p);
}

hipError_t pinned_alloc(void** p, size_t bytes, size_t* got) {
  if (bytes == 0) bytes = 1;
  if (bytes >= kMinCached) {
    if (void* q = pinned_cache().take(bytes, 0, got)) {
      *p = q;
      return hipSuccess;
    }
  }
  *got = bytes;
  return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

void pinned_free(void* p, size_t bytes) {
  if (!p) return;
  // every copy into a batch buffer is waited for by its owner (fetch_span,
  // the batch prefetch): no device-wide wait here
  if (bytes >= kMinCached && pinned_cache().put(p, bytes, 0, kPinnedCap)) return;
  (void)hipHostFree(p);
}

size_t release_cached() {
  std::multimap<size_t, std::pair<void*, int>> d, h;
  size_t n = dev_cache().drain(&d) + pinned_cache().drain(&h);
  const int cur = current_device();
  for (auto& b : d) {
    (void)hipSetDevice(b.second.second);
    (void)hipFree(b.second.first);
  }
  if (cur >= 0) (void)hipSetDevice(cur);
  for (auto& b : h) (void)hipHostFree(b.second.first);
  return n;
}

}  // namespace hbam
