// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE for the access
// shapes of the record kernels (developer probe, not product).
// MI355X_MICROARCH.md: FETCH_SIZE is exactly 1/2 of the bytes of a wide
// coalesced streaming read on gfx950; "other access widths are uncalibrated".
// The walk and the fused check read a few dwords per ~340 B record, so the
// bench's traffic of those kernels needs the factor for sparse reads.  Each
// kernel below reads a 4 GiB buffer (past the 256 MiB Infinity Cache) in one
// shape; the printed "lines" is the number of distinct 128 B lines it
// touches.  Run: rocprofv3 --pmc FETCH_SIZE -- scripts/bin/fetch_calib
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/bin/fetch_calib scripts/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// 16 B per lane, consecutive (the guide's calibrated case)
__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads
}

// one dword per `stride` bytes (lanes `stride` apart)
__global__ void k_sparse4(const uint8_t* __restrict__ a, uint64_t bytes, uint32_t stride, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint64_t n = bytes / stride;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= *reinterpret_cast<const uint32_t*>(a + i * stride);
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// 40 B (a record head: 2 x 16 B + 8 B) per `stride` bytes at an offset that
// walks through its 128 B line (4 B aligned; stride a multiple of 128)
__global__ void k_sparse_head(const uint8_t* __restrict__ a, uint64_t bytes, uint32_t stride,
                              uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint64_t n = bytes / stride - 1;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q = i * stride + ((i * 36) & 0x7c);
    const uint32_t* p = reinterpret_cast<const uint32_t*>(a + q);
#pragma unroll
    for (int k = 0; k < 10; ++k) acc ^= p[k];
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 4ull << 30;
  uint8_t* a = nullptr;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&a, bytes + 4096));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(a, 1, bytes + 4096));
  CHK(hipDeviceSynchronize());
  const int grid = 8192, block = 256;
  hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(block), 0, 0, reinterpret_cast<const uint4*>(a), bytes / 16, out);
  printf("k_stream16: %llu bytes read, %llu lines\n", (unsigned long long)bytes, (unsigned long long)(bytes / 128));
  for (uint32_t stride : {128u, 256u, 340u, 512u}) {
    hipLaunchKernelGGL(k_sparse4, dim3(grid), dim3(block), 0, 0, a, bytes, stride, out);
    printf("k_sparse4 stride %u: %llu dwords, %llu lines\n", stride, (unsigned long long)(bytes / stride),
           (unsigned long long)(bytes / stride));
  }
  for (uint32_t stride : {384u}) {
    hipLaunchKernelGGL(k_sparse_head, dim3(grid), dim3(block), 0, 0, a, bytes, stride, out);
    // lines touched per record: the 40 B at offset (i*36)&0x7c inside its 128 B-aligned slot straddles
    // into the next line when that offset > 88 (offsets 92..124: 9 of 32 values)
    printf("k_sparse_head stride %u: %llu records, ~%.0f lines\n", stride, (unsigned long long)(bytes / stride),
           (double)(bytes / stride) * (1.0 + 9.0 / 32.0));
  }
  CHK(hipDeviceSynchronize());
  CHK(hipFree(a));
  CHK(hipFree(out));
  return 0;
}
