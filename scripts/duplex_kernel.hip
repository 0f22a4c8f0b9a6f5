// Developer probe (scripts/duplex_probe.py --kernel): a host->HBM copy done by
// a kernel that loads page-locked host memory, to run beside an SDMA HBM->host
// copy.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/_duplex.so scripts/duplex_kernel.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

struct alignas(16) V4 {
  uint32_t x, y, z, w;
};

__global__ void __launch_bounds__(256) k_pull(const V4* __restrict__ src, V4* __restrict__ dst, uint64_t n16) {
  constexpr int kU = 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (kU - 1) * stride < n16; i += kU * stride) {
    V4 v[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) v[k] = src[i + k * stride];
#pragma unroll
    for (int k = 0; k < kU; ++k) dst[i + k * stride] = v[k];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

extern "C" int duplex_pull(const void* host_src, void* dst, uint64_t bytes, int blocks, void* stream) {
  void* dsrc = nullptr;
  if (hipHostGetDevicePointer(&dsrc, const_cast<void*>(host_src), 0) != hipSuccess) return -1;
  if (bytes % 16) return -2;
  hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const V4*)dsrc, (V4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
