// h2d_map_probe.hip -- host -> HBM feeds of a file in /dev/shm (developer
// probe): what a fresh mmap costs per path.  Each case maps the file anew.
//   pageable      hipMemcpy from the mapping (cold), then again (warm)
//   register      hipHostRegister of the mapping (T threads over sub-ranges),
//                 then hipMemcpy from it
//   pread->pinned T threads pread() 64 MiB pieces into two page-locked
//                 buffers, each piece copied to HBM while the next is read
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/h2d_map_probe scripts/h2d_map_probe.hip -lpthread
// Usage: h2d_map_probe <file>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                              \
    }                                                        \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  fstat(fd, &st);
  const size_t n = st.st_size;
  void* d;
  CK(hipMalloc(&d, n));
  auto map = [&]() { return (uint8_t*)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0); };
  // pageable, cold then warm
  {
    uint8_t* m = map();
    double t = now();
    CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
    double a = now() - t;
    t = now();
    CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
    double b = now() - t;
    printf("pageable: cold %.1f ms (%.1f GB/s), warm %.1f ms (%.1f GB/s)\n", a * 1e3, n / a / 1e9, b * 1e3,
           n / b / 1e9);
    munmap(m, n);
  }
  for (int T : {1, 4, 8, 16}) {
    uint8_t* m = map();
    double t = now();
    std::vector<std::thread> th;
    const size_t page = 4096, per = ((n + T - 1) / T + page - 1) / page * page;
    std::vector<hipError_t> es(T, hipSuccess);
    for (int i = 0; i < T; ++i)
      th.emplace_back([&, i]() {
        size_t lo = i * per, hi = std::min(n, lo + per);
        if (lo < hi) es[i] = hipHostRegister(m + lo, hi - lo, hipHostRegisterReadOnly);
      });
    for (auto& x : th) x.join();
    double a = now() - t;
    for (auto e : es) CK(e);
    t = now();
    for (int i = 0; i < T; ++i) {  // a copy may not span two registrations
      size_t lo = i * per, hi = std::min(n, lo + per);
      if (lo < hi) CK(hipMemcpyAsync((uint8_t*)d + lo, m + lo, hi - lo, hipMemcpyHostToDevice, 0));
    }
    CK(hipDeviceSynchronize());
    double b = now() - t;
    printf("register x%d: register %.1f ms, copy %.1f ms (%.1f GB/s), both %.1f GB/s\n", T, a * 1e3, b * 1e3,
           n / b / 1e9, n / (a + b) / 1e9);
    for (int i = 0; i < T; ++i) {
      size_t lo = i * per;
      if (lo < n) (void)hipHostUnregister(m + lo);
    }
    munmap(m, n);
  }
  for (int T : {4, 8, 16}) {  // cold pageable copies of sub-ranges from T threads at once
    uint8_t* m = map();
    const size_t per = (n + T - 1) / T;
    double t = now();
    std::vector<std::thread> th;
    std::vector<hipError_t> es(T, hipSuccess);
    for (int i = 0; i < T; ++i)
      th.emplace_back([&, i]() {
        size_t lo = i * per, hi = std::min(n, lo + per);
        hipStream_t s;
        es[i] = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        if (es[i] == hipSuccess && lo < hi) es[i] = hipMemcpyAsync((uint8_t*)d + lo, m + lo, hi - lo, hipMemcpyHostToDevice, s);
        if (es[i] == hipSuccess) es[i] = hipStreamSynchronize(s);
      });
    for (auto& x : th) x.join();
    double a = now() - t;
    for (auto e : es) CK(e);
    printf("pageable x%d threads (cold): %.1f ms (%.1f GB/s)\n", T, a * 1e3, n / a / 1e9);
    munmap(m, n);
  }
  for (int T : {4, 8, 16}) {  // T threads memcpy a fresh mapping into page-locked pieces
    const size_t piece = 64ull << 20;
    uint8_t* m = map();
    uint8_t* pin[2];
    CK(hipHostMalloc((void**)&pin[0], piece, 0));
    CK(hipHostMalloc((void**)&pin[1], piece, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev[2];
    CK(hipEventCreate(&ev[0]));
    CK(hipEventCreate(&ev[1]));
    double t = now();
    for (size_t o = 0, k = 0; o < n; o += piece, ++k) {
      const size_t len = std::min(piece, n - o);
      uint8_t* b = pin[k & 1];
      if (k >= 2) CK(hipEventSynchronize(ev[k & 1]));
      std::vector<std::thread> th;
      const size_t per = (len + T - 1) / T;
      for (int i = 0; i < T; ++i)
        th.emplace_back([&, i]() {
          size_t lo = i * per, hi = std::min(len, lo + per);
          if (lo < hi) memcpy(b + lo, m + o + lo, hi - lo);
        });
      for (auto& x : th) x.join();
      CK(hipMemcpyAsync((uint8_t*)d + o, b, len, hipMemcpyHostToDevice, s));
      CK(hipEventRecord(ev[k & 1], s));
    }
    CK(hipStreamSynchronize(s));
    double a = now() - t;
    printf("mmap memcpy->pinned x%d: %.1f ms (%.1f GB/s)\n", T, a * 1e3, n / a / 1e9);
    (void)hipHostFree(pin[0]);
    (void)hipHostFree(pin[1]);
    munmap(m, n);
  }
  for (int T : {4, 8, 16}) {
    const size_t piece = 64ull << 20;
    uint8_t* pin[2];
    CK(hipHostMalloc((void**)&pin[0], piece, 0));
    CK(hipHostMalloc((void**)&pin[1], piece, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev[2];
    CK(hipEventCreate(&ev[0]));
    CK(hipEventCreate(&ev[1]));
    double t = now();
    for (size_t o = 0, k = 0; o < n; o += piece, ++k) {
      const size_t len = std::min(piece, n - o);
      uint8_t* b = pin[k & 1];
      if (k >= 2) CK(hipEventSynchronize(ev[k & 1]));
      std::vector<std::thread> th;
      const size_t per = (len + T - 1) / T;
      for (int i = 0; i < T; ++i)
        th.emplace_back([&, i]() {
          size_t lo = i * per, hi = std::min(len, lo + per);
          while (lo < hi) {
            ssize_t r = pread(fd, b + lo, hi - lo, o + lo);
            if (r <= 0) break;
            lo += r;
          }
        });
      for (auto& x : th) x.join();
      CK(hipMemcpyAsync((uint8_t*)d + o, b, len, hipMemcpyHostToDevice, s));
      CK(hipEventRecord(ev[k & 1], s));
    }
    CK(hipStreamSynchronize(s));
    double a = now() - t;
    printf("pread->pinned x%d: %.1f ms (%.1f GB/s)\n", T, a * 1e3, n / a / 1e9);
    (void)hipHostFree(pin[0]);
    (void)hipHostFree(pin[1]);
  }
  return 0;
}
