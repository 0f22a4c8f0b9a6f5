// sdma_probe.hip -- do small copies on one stream wait behind a large
// device->host copy on another (developer probe)?  Times, while a 1 GiB
// D2H (page-locked) runs on stream A: an 8-byte D2H on stream B, an 8-byte
// pageable H2D on stream B, and an 8-byte read-back by a kernel writing into
// page-locked memory on stream B.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/bin/sdma_probe scripts/sdma_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void k_read(unsigned long long* dst, const unsigned long long* src) { *dst = *src; }
__global__ void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t big = 1ull << 30;
  void *dbig, *hbig, *dsmall;
  unsigned long long* hsmall;
  CK(hipMalloc(&dbig, big));
  CK(hipHostMalloc(&hbig, big, hipHostMallocDefault));
  CK(hipMalloc(&dsmall, 64));
  CK(hipHostMalloc((void**)&hsmall, 64, hipHostMallocDefault));
  CK(hipMemset(dbig, 1, big));
  CK(hipMemset(dsmall, 2, 64));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 6; ++mode) {
      double t0 = now_ms();
      if (mode > 0) CK(hipMemcpyAsync(hbig, dbig, big, hipMemcpyDeviceToHost, a));
      double t1 = now_ms();
      unsigned long long v = 0;
      const char* what = "";
      if (mode == 0 || mode == 1) {
        CK(hipMemcpyAsync(hsmall, dsmall, 8, hipMemcpyDeviceToHost, b));
        what = mode == 0 ? "8 B D2H alone" : "8 B D2H (pinned) beside 1 GiB D2H";
      } else if (mode == 2) {
        CK(hipMemcpyAsync(dsmall, &v, 8, hipMemcpyHostToDevice, b));
        what = "8 B pageable H2D beside 1 GiB D2H";
      } else if (mode == 4) {
        CK(hipMemcpyAsync(&v, dsmall, 8, hipMemcpyDeviceToHost, b));
        what = "8 B D2H into pageable beside 1 GiB D2H";
      } else if (mode == 5) {
        CK(hipMemcpy(&v, dsmall, 8, hipMemcpyDeviceToHost));
        what = "8 B sync hipMemcpy D2H beside 1 GiB D2H";
      } else {
        k_read<<<1, 1, 0, b>>>(hsmall, (const unsigned long long*)dsmall);
        CK(hipGetLastError());
        what = "8 B kernel read-back beside 1 GiB D2H";
      }
      CK(hipStreamSynchronize(b));
      double t2 = now_ms();
      CK(hipStreamSynchronize(a));
      double t3 = now_ms();
      printf("rep %d %-40s small done after %7.3f ms, big done after %7.3f ms (issue %.3f)\n", rep, what, t2 - t1,
             t3 - t1, t1 - t0);
    }
  }
  // full duplex?  a 1 GiB H2D (page-locked) beside a 1 GiB D2H, both by copy
  // engines, then the D2H by a kernel writing page-locked memory
  void *hbig2, *dbig2;
  CK(hipHostMalloc(&hbig2, big, hipHostMallocDefault));
  CK(hipMalloc(&dbig2, big));
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now_ms();
    CK(hipMemcpyAsync(dbig2, hbig2, big, hipMemcpyHostToDevice, b));
    CK(hipStreamSynchronize(b));
    double t1 = now_ms();
    CK(hipMemcpyAsync(hbig, dbig, big, hipMemcpyDeviceToHost, a));
    CK(hipMemcpyAsync(dbig2, hbig2, big, hipMemcpyHostToDevice, b));
    CK(hipStreamSynchronize(b));
    double t2 = now_ms();
    CK(hipStreamSynchronize(a));
    double t3 = now_ms();
    printf("H2D alone %.2f ms; H2D beside D2H: H2D %.2f ms, both %.2f ms\n", t1 - t0, t2 - t1, t3 - t1);
    for (int wg : {16, 32, 64, 128}) {
      double u0 = now_ms();
      k_copy<<<wg, 256, 0, a>>>((uint4*)hbig, (const uint4*)dbig, big / 16);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(a));
      double u1 = now_ms();
      k_copy<<<wg, 256, 0, a>>>((uint4*)hbig, (const uint4*)dbig, big / 16);
      CK(hipMemcpyAsync(dbig2, hbig2, big, hipMemcpyHostToDevice, b));
      CK(hipStreamSynchronize(b));
      double u2 = now_ms();
      CK(hipStreamSynchronize(a));
      double u3 = now_ms();
      printf("  kernel D2H (%d WG) alone %.2f ms (%.1f GB/s); beside SDMA H2D: H2D %.2f ms, both %.2f ms\n", wg,
             u1 - u0, big / (u1 - u0) / 1e6, u2 - u1, u3 - u1);
    }
  }
  return 0;
}
