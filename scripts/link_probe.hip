// link_probe.hip -- is the host link full duplex, and through which engine?
// (scripts/ probe for the drop-in batch path; not product code)
//   hipcc --offload-arch=gfx950 -O2 -o scripts/bin/link_probe scripts/link_probe.hip
// Measures 1 GiB transfers: SDMA D2H / H2D alone and together; a kernel
// that streams device memory into mapped page-locked host memory (D2H by
// the shader) and one that reads host memory into HBM (H2D), each alone and
// beside the opposite SDMA copy.  Prints GB/s per direction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static double run(hipStream_t* s, int ns, void (*issue)(int, hipStream_t), int reps = 3) {
  double best = 1e30;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < reps; ++r) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, nullptr));
    for (int i = 0; i < ns; ++i) {
      CK(hipStreamWaitEvent(s[i], a, 0));
      issue(i, s[i]);
    }
    for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(s[i]));
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

static const size_t N = 1ull << 30;
static uint8_t *d_a, *d_b, *h_a, *h_b, *h_a_dev, *h_b_dev;
static int g_mode[2];
// modes: 0 SDMA D2H (d_a -> h_a), 1 SDMA H2D (h_b -> d_b), 2 kernel D2H, 3 kernel H2D
static void issue(int i, hipStream_t s) {
  switch (g_mode[i]) {
    case 0: CK(hipMemcpyAsync(h_a, d_a, N, hipMemcpyDeviceToHost, s)); break;
    case 1: CK(hipMemcpyAsync(d_b, h_b, N, hipMemcpyHostToDevice, s)); break;
    case 2:
      hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s, (const uint4*)d_a, (uint4*)h_a_dev, N / 16);
      break;
    case 3:
      hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s, (const uint4*)h_b_dev, (uint4*)d_b, N / 16);
      break;
  }
}

int main() {
  CK(hipMalloc(&d_a, N));
  CK(hipMalloc(&d_b, N));
  CK(hipMemset(d_a, 1, N));
  CK(hipHostMalloc(&h_a, N, hipHostMallocMapped));
  CK(hipHostMalloc(&h_b, N, hipHostMallocMapped));
  memset(h_b, 2, N);
  CK(hipHostGetDevicePointer((void**)&h_a_dev, h_a, 0));
  CK(hipHostGetDevicePointer((void**)&h_b_dev, h_b, 0));
  hipStream_t s[2];
  CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
  const char* names[4] = {"sdma_d2h", "sdma_h2d", "kernel_d2h", "kernel_h2d"};
  printf("{");
  for (int m = 0; m < 4; ++m) {
    g_mode[0] = m;
    double ms = run(s, 1, issue);
    printf("\"%s\": %.2f, ", names[m], N / ms / 1e6);
  }
  int pairs[4][2] = {{0, 1}, {2, 1}, {0, 3}, {2, 3}};
  for (int p = 0; p < 4; ++p) {
    g_mode[0] = pairs[p][0];
    g_mode[1] = pairs[p][1];
    double ms = run(s, 2, issue);
    printf("\"%s+%s_each\": %.2f%s", names[pairs[p][0]], names[pairs[p][1]], N / ms / 1e6, p < 3 ? ", " : "");
  }
  printf("}\n");
  return 0;
}
