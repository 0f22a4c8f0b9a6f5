// hbam_mem.h -- process-wide caches of device and page-locked host blocks.
//
// Every split a JVM opens (hbam_open -> hbam_decode_span, BAMRecordReader.
// initialize / nextKeyValue) builds a pipeline whose buffers run to
// gigabytes: ~1.4x the window in HBM and the batch columns + record bytes in
// page-locked host memory.  Allocating and pinning them per split costs more
// than decoding a C2 split (hipHostMalloc of a 1M-record batch, ~0.3 s).  A
// freed block goes back to a per-process cache instead and the next split of
// the same process (a Spark executor or a reused task JVM reads many) takes
// it.
//
// Concurrency: many contexts (one per reader thread of an executor) share a
// GPU.  A released block may still be read by work its owner queued, so the
// owner waits for ITS streams (StreamSet) before a block is released or
// handed on -- never for the whole device, which would stall every other
// reader on the GPU.  The caches themselves are mutex-guarded.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace hbam {

// The streams whose queued work may touch an owner's blocks.
struct StreamSet {
  hipStream_t s[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  int n = 0;
  hipError_t sync() const {
    for (int i = 0; i < n; ++i)
      if (s[i]) {
        const hipError_t e = hipStreamSynchronize(s[i]);
        if (e != hipSuccess) return e;
      }
    return hipSuccess;
  }
};

// A block of at least `bytes` on the current device (a cached one of at most
// twice the size, else hipMalloc); *got = its size.
hipError_t dev_alloc(void** p, size_t bytes, size_t* got);
// The caller has waited for every stream that used the block.
void dev_free(void* p, size_t bytes);

// Page-locked host memory (hipHostMalloc), cached the same way; the caller
// has waited for every copy into or out of the block before freeing it.
hipError_t pinned_alloc(void** p, size_t bytes, size_t* got);
void pinned_free(void* p, size_t bytes);

// Every cached block back to the HIP runtime; returns the bytes released.
size_t release_cached();

}  // namespace hbam
