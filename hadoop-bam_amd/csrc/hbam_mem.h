// hbam_mem.h -- process-wide caches of device and page-locked host blocks.
//
// Every split a JVM opens (hbam_open -> hbam_decode_span, BAMRecordReader.
// initialize / nextKeyValue) builds a pipeline whose buffers run to
// gigabytes: ~1.4x the window in HBM and the batch columns + record bytes in
// page-locked host memory.  Allocating and pinning them per split costs more
// than decoding a C2 split (hipHostMalloc of a 1M-record batch, ~0.3 s).  A
// freed block goes back to a per-process cache instead and the next split of
// the same process (a Spark executor or a reused task JVM reads many) takes
// it.  A released block may still be read by queued work, so the device is
// synchronized first, as hipFree / hipHostFree would.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace hbam {

// A block of at least `bytes` on the current device (a cached one of at most
// twice the size, else hipMalloc); *got = its size.
hipError_t dev_alloc(void** p, size_t bytes, size_t* got);
void dev_free(void* p, size_t bytes);

// Page-locked host memory (hipHostMalloc), cached the same way.
hipError_t pinned_alloc(void** p, size_t bytes, size_t* got);
void pinned_free(void* p, size_t bytes);

// Every cached block back to the HIP runtime; returns the bytes released.
size_t release_cached();

}  // namespace hbam
