// hbam_deflate.hip -- BGZF write path on the GPU: [htsjdk]
// BlockCompressedOutputStream.deflateBlock + writeGzipBlock for every block
// of a payload stream at once (the compressor behind BAMRecordWriter /
// KeyIgnoringBAMRecordWriter output, BAMRecordWriter.java:131-149).
//
//   k_deflate_blocks  one lane per BGZF block: zlib 1.2.11 deflate_fast
//                     (levels 1-3) / deflate_slow (4-9) + trees.c restated in hbam_deflate.h (byte-identical
//                     output), hash chains / symbol buffer / trees in a
//                     per-lane arena in HBM, cdata into a 64 KiB slot.
//   k_dfl_crc         one 1024-thread workgroup per block: CRC-32 of the
//                     payload (64-byte parts, slice-by-8, combined pairwise).
//   k_dfl_frame       one workgroup per block: 18-byte BGZF header, cdata
//                     (or htsjdk's level-0 fallback: one stored block) and
//                     the CRC32 / ISIZE footer at the block's file offset.
// Deflate is a serial recurrence within a block (lazy matching over hash
// chains), so parallelism is across blocks; the host only turns the per-block
// sizes into file offsets.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "hbam_deflate.h"
#include "hbam_deflate_api.h"

namespace hbam {

namespace {

constexpr uint32_t kSlot = 65536;      // cdata slot per block
constexpr uint32_t kMaxLanes = 65536;  // concurrent arenas (~184 KiB each)
constexpr uint32_t kCrcPoly = 0xedb88320u;
constexpr uint32_t kWavesTarget = 5120;  // 5 waves per SIMD (84 VGPRs: occupancy 5; measured best)

__device__ inline uint32_t crc_mul(uint32_t a, uint32_t b) {  // a * b mod P (reflected)
  if (a == 0) return 0;
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

__global__ __launch_bounds__(64) void k_deflate_blocks(const uint8_t* __restrict__ in, const uint64_t* __restrict__ ustart,
                                                       const uint32_t* __restrict__ lens, uint32_t b0, uint32_t nb,
                                                       int level, const dfl::Tables* __restrict__ tables,
                                                       dfl::Arena* __restrict__ arenas, uint8_t* __restrict__ slots,
                                                       uint32_t* __restrict__ csize, uint8_t* __restrict__ ovf,
                                                       uint32_t lpw) {
  // lpw active lanes per wave: the work is a serial, latency-bound recurrence
  // per lane, so spreading blocks over more SIMDs (and fewer divergent lanes
  // per wave) beats packing 64 lanes into one wave
  if (threadIdx.x >= lpw) return;
  const uint32_t i = blockIdx.x * lpw + threadIdx.x;
  if (i >= nb) return;
  const uint32_t b = b0 + i;
  dfl::Arena* a = arenas + i;
  uint4* h = reinterpret_cast<uint4*>(a->head);
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int k = 0; k < (int)(sizeof(a->head) / 16); ++k) h[k] = z;
  bool o = false;
  if (level == 0) {  // Deflater(NO_COMPRESSION): one stored block, written by k_dfl_frame
    csize[b] = 0;
    ovf[b] = 1;
    return;
  }
  const uint32_t n = dfl::deflate_block(a, tables, level, in + ustart[b], lens[b], slots + (uint64_t)i * kSlot,
                                        dfl::kOutCap, &o, true);
  csize[b] = n;
  ovf[b] = o ? 1 : 0;
}

// CRC-32 (zlib crc32) of each block's payload.  1024 threads per block: the
// payload is viewed as front-padded with zeros to 64 KiB (a raw CRC -- zero
// initial state -- ignores leading zeros; zlib's ~0 initial state is the
// same as complementing the first four bytes), so thread t owns the 64 bytes
// [64t, 64t + 64) of that view and every part has the same length: the parts
// are combined pairwise in 10 rounds, round k multiplying by the constant
// x^(8*64*2^k) mod P.  Each part is computed slice-by-8 from LDS tables; the
// tables and multipliers are built once on the host (crc_constants).
constexpr uint32_t kCrcThreads = 1024;
constexpr uint32_t kCrcPart = 65536 / kCrcThreads;  // bytes per thread
constexpr uint32_t kCrcRounds = 10;                  // log2(kCrcThreads)
constexpr uint32_t kCrcConstWords = 8 * 256 + kCrcRounds;

__global__ __launch_bounds__(1024) void k_dfl_crc(const uint8_t* __restrict__ in, const uint64_t* __restrict__ ustart,
                                                  const uint32_t* __restrict__ lens,
                                                  const uint32_t* __restrict__ consts, uint32_t* __restrict__ crc) {
  __shared__ uint32_t tab[8][256];
  __shared__ uint32_t part[kCrcThreads];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  const uint32_t len = lens[b];
  const uint8_t* p = in + ustart[b];
  for (uint32_t i = t; i < 8 * 256; i += kCrcThreads) (&tab[0][0])[i] = consts[i];
  __syncthreads();
  if (len < 4) {  // too short for the complement form: one thread, byte by byte
    if (t == 0) {
      uint32_t r = 0xffffffffu;
      for (uint32_t i = 0; i < len; ++i) r = tab[0][(r ^ p[i]) & 0xff] ^ (r >> 8);
      crc[b] = r ^ 0xffffffffu;
    }
    return;
  }
  // this thread's bytes of the payload: [64t - pad, 64t + 64 - pad) clipped to [0, len)
  const int64_t pad = 65536 - (int64_t)len;
  const int64_t r0 = max<int64_t>(0, (int64_t)kCrcPart * t - pad);
  const int64_t r1 = max<int64_t>(0, (int64_t)kCrcPart * (t + 1) - pad);
  uint32_t r = 0;
  int64_t i = r0;
  for (; i + 8 <= r1; i += 8) {
    uint64_t v = dfl::ld8(p + i);
    if (i < 4) v ^= (uint64_t)(0xffffffffu >> (8 * i));  // the initial ~0: payload bytes i..3
    const uint32_t lo = (uint32_t)v ^ r, hi = (uint32_t)(v >> 32);
    r = tab[7][lo & 0xff] ^ tab[6][(lo >> 8) & 0xff] ^ tab[5][(lo >> 16) & 0xff] ^ tab[4][lo >> 24] ^
        tab[3][hi & 0xff] ^ tab[2][(hi >> 8) & 0xff] ^ tab[1][(hi >> 16) & 0xff] ^ tab[0][hi >> 24];
  }
  for (; i < r1; ++i) r = tab[0][(r ^ p[i] ^ (i < 4 ? 0xffu : 0u)) & 0xff] ^ (r >> 8);
  part[t] = r;
  __syncthreads();
  for (uint32_t k = 0, s = 1; s < kCrcThreads; ++k, s <<= 1) {  // pairwise combine
    if ((t & (2 * s - 1)) == 0) part[t] = crc_mul(consts[8 * 256 + k], part[t]) ^ part[t + s];
    __syncthreads();
  }
  if (t == 0) crc[b] = part[0] ^ 0xffffffffu;
}

// Host: the slice-by-8 tables and x^(8*64*2^k) mod P, k < kCrcRounds.
static uint32_t host_crc_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
static std::vector<uint32_t> crc_constants() {
  std::vector<uint32_t> c(kCrcConstWords);
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t v = n;
    for (int k = 0; k < 8; ++k) v = (v & 1) ? (v >> 1) ^ kCrcPoly : v >> 1;
    c[n] = v;
  }
  for (uint32_t k = 1; k < 8; ++k)
    for (uint32_t n = 0; n < 256; ++n) c[256 * k + n] = (c[256 * (k - 1) + n] >> 8) ^ c[c[256 * (k - 1) + n] & 0xff];
  uint32_t x = 1u << 30;  // x^1
  for (int k = 0; k < 3; ++k) x = host_crc_mul(x, x);  // x^8
  uint32_t xp = 1u << 31;  // x^(8 * kCrcPart)
  for (uint32_t n = kCrcPart; n; n >>= 1, x = host_crc_mul(x, x))
    if (n & 1) xp = host_crc_mul(x, xp);
  for (uint32_t k = 0; k < kCrcRounds; ++k, xp = host_crc_mul(xp, xp)) c[8 * 256 + k] = xp;
  return c;
}

// BGZF framing ([htsjdk] BlockCompressedOutputStream.writeGzipBlock)
__global__ __launch_bounds__(256) void k_dfl_frame(const uint8_t* __restrict__ in, const uint64_t* __restrict__ ustart,
                                                   const uint32_t* __restrict__ lens,
                                                   const uint8_t* __restrict__ slots,
                                                   const uint32_t* __restrict__ csize, const uint8_t* __restrict__ ovf,
                                                   const uint32_t* __restrict__ crc, const uint64_t* __restrict__ offs,
                                                   uint8_t* __restrict__ out, uint32_t b0) {
  const uint32_t b = b0 + blockIdx.x;  // slots hold the current batch only
  const uint32_t len = lens[b];
  const bool stored = ovf[b] != 0;
  const uint32_t cn = stored ? len + 5 : csize[b];
  uint8_t* o = out + offs[b];
  const uint32_t total = cn + 26;
  if (threadIdx.x < 18) {
    const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
    const uint32_t t = threadIdx.x;
    o[t] = t < 16 ? hdr[t] : (uint8_t)((total - 1) >> (8 * (t - 16)));
  } else if (threadIdx.x < 26) {
    const uint32_t t = threadIdx.x - 18;
    o[18 + cn + t] = (uint8_t)((t < 4 ? crc[b] : len) >> (8 * (t & 3)));
  }
  uint8_t* c = o + 18;
  if (!stored) {
    const uint8_t* s = slots + (uint64_t)blockIdx.x * kSlot;
    for (uint32_t i = threadIdx.x; i < cn; i += 256) c[i] = s[i];
  } else {  // Deflater(NO_COMPRESSION): one final stored block
    if (threadIdx.x == 0) {
      c[0] = 1;
      c[1] = (uint8_t)len;
      c[2] = (uint8_t)(len >> 8);
      c[3] = (uint8_t)~len;
      c[4] = (uint8_t)(~len >> 8);
    }
    const uint8_t* s = in + ustart[b];
    for (uint32_t i = threadIdx.x; i < len; i += 256) c[5 + i] = s[i];
  }
}

}  // namespace

#define DCHK(x)                                                   \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      err_ = std::string(#x) + ": " + hipGetErrorString(e_);      \
      return kDeviceErr;                                          \
    }                                                             \
  } while (0)

BgzfCompressor::BgzfCompressor(int device) : device_(device) {}

BgzfCompressor::~BgzfCompressor() {
  for (void* p : {(void*)tables_, (void*)arenas_, (void*)slots_, (void*)csize_, (void*)ovf_, (void*)crc_,
                  (void*)offs_, (void*)out_, (void*)ustart_, (void*)lens_, (void*)crc_tab_})
    if (p) (void)hipFree(p);
}

template <typename T>
static hipError_t grow_buf(T** p, size_t* have, size_t need, hipStream_t s) {
  if (*p && *have >= need) return hipSuccess;
  if (*p) {
    (void)hipStreamSynchronize(s);  // the compressor's work runs on s only
    (void)hipFree(*p);
  }
  *p = nullptr;
  *have = 0;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), need ? need : 1);
  if (e == hipSuccess) *have = need;
  return e;
}

int BgzfCompressor::compress(const uint8_t* d_in, const std::vector<uint64_t>& ustart,
                             const std::vector<uint32_t>& lens, int level, bool eof, hipStream_t s, float* ms) {
  const int kDeviceErr = 5, kArgErr = 3, kFormatErr = 1;
  if (level < 0 || level > 9) {
    err_ = "level must be 0..9 (htsjdk default 5)";
    return kArgErr;
  }
  const uint64_t nb = lens.size();
  for (uint32_t l : lens)
    if (l > 65536) {
      err_ = "BGZF payload above 65536 bytes";
      return kArgErr;
    }
  out_len_ = 0;
  fallbacks_ = 0;
  DCHK(hipSetDevice(device_));
  if (!crc_tab_) {
    const std::vector<uint32_t> c = crc_constants();
    DCHK(hipMalloc(reinterpret_cast<void**>(&crc_tab_), c.size() * 4));
    DCHK(hipMemcpy(crc_tab_, c.data(), c.size() * 4, hipMemcpyHostToDevice));
  }
  if (!tables_) {
    dfl::Tables t;
    dfl::build_tables(&t);
    DCHK(hipMalloc(reinterpret_cast<void**>(&tables_), sizeof t));
    DCHK(hipMemcpy(tables_, &t, sizeof t, hipMemcpyHostToDevice));
  }
  // Blocks go through in batches of up to kMaxLanes: deflate (a lane and an
  // arena per block, cdata into the batch's slots), sizes to the host, file
  // offsets continued from the previous batch, framing.  Memory is bounded by
  // one batch's arenas + slots whatever the stream length; the output is
  // sized for the worst case: a compressed block is never larger than its
  // stored form (len + 5 B per DEFLATE block, <= 5 blocks of 16,383 symbols),
  // the fallback is len + 5, plus 26 B of framing.
  const char* ml = getenv("HBAM_DFL_MAX_LANES");  // test knob: force several batches
  const uint64_t max_lanes = ml ? (uint64_t)std::max(1, atoi(ml)) : kMaxLanes;
  const uint32_t lanes = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(nb, 1), max_lanes);
  uint64_t worst = eof ? 28 : 0;
  for (uint32_t l : lens) worst += (uint64_t)l + 26 + 64;
  DCHK(grow_buf(&arenas_, &arenas_n_, (size_t)lanes * sizeof(dfl::Arena), s));
  DCHK(grow_buf(&slots_, &slots_n_, (size_t)lanes * kSlot, s));
  DCHK(grow_buf(&csize_, &csize_n_, std::max<uint64_t>(nb, 1) * 4, s));
  DCHK(grow_buf(&ovf_, &ovf_n_, std::max<uint64_t>(nb, 1), s));
  DCHK(grow_buf(&crc_, &crc_n_, std::max<uint64_t>(nb, 1) * 4, s));
  DCHK(grow_buf(&offs_, &offs_n_, (nb + 1) * 8, s));
  DCHK(grow_buf(&ustart_, &ustart_n_, std::max<uint64_t>(nb, 1) * 8, s));
  DCHK(grow_buf(&lens_, &lens_n_, std::max<uint64_t>(nb, 1) * 4, s));
  DCHK(grow_buf(&out_, &out_n_, worst + 16, s));
  struct Ev {  // destroyed on every return path
    hipEvent_t e = nullptr;
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev0, ev1;
  DCHK(hipEventCreate(&ev0.e));
  DCHK(hipEventCreate(&ev1.e));
  const hipEvent_t e0 = ev0.e, e1 = ev1.e;
  DCHK(hipEventRecord(e0, s));
  std::vector<uint32_t> cs(nb);
  std::vector<uint8_t> ov(nb);
  std::vector<uint64_t> offs(nb + 1);
  uint64_t o = 0;
  if (nb) {
    DCHK(hipMemcpyAsync(ustart_, ustart.data(), nb * 8, hipMemcpyHostToDevice, s));
    DCHK(hipMemcpyAsync(lens_, lens.data(), nb * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_dfl_crc, dim3((uint32_t)nb), dim3(kCrcThreads), 0, s, d_in, ustart_, lens_, crc_tab_,
                       crc_);
    DCHK(hipGetLastError());
    const uint32_t waves = kWavesTarget;
    for (uint64_t b0 = 0; b0 < nb; b0 += lanes) {
      const uint32_t n = (uint32_t)std::min<uint64_t>(lanes, nb - b0);
      // about kWavesTarget waves in flight over 256 CUs x 4 SIMDs
      const uint32_t lpw = std::max<uint32_t>(1, std::min<uint32_t>(64, (n + waves - 1) / waves));
      hipLaunchKernelGGL(k_deflate_blocks, dim3((n + lpw - 1) / lpw), dim3(64), 0, s, d_in, ustart_, lens_,
                         (uint32_t)b0, n, level, tables_, arenas_, slots_, csize_, ovf_, lpw);
      DCHK(hipGetLastError());
      DCHK(hipMemcpyAsync(cs.data() + b0, csize_ + b0, (size_t)n * 4, hipMemcpyDeviceToHost, s));
      DCHK(hipMemcpyAsync(ov.data() + b0, ovf_ + b0, n, hipMemcpyDeviceToHost, s));
      DCHK(hipStreamSynchronize(s));
      for (uint64_t b = b0; b < b0 + n; ++b) {
        offs[b] = o;
        if (ov[b] && lens[b] + 5 > dfl::kOutCap) {
          err_ = "incompressible BGZF payload does not fit one stored block";
          return kFormatErr;
        }
        o += 26 + (ov[b] ? lens[b] + 5 : cs[b]);
      }
      if (o + (eof ? 28 : 0) > worst) {  // cannot happen (see the bound above); never write past out_
        err_ = "BGZF output bound exceeded";
        return kFormatErr;
      }
      DCHK(hipMemcpyAsync(offs_ + b0, offs.data() + b0, (size_t)n * 8, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_dfl_frame, dim3(n), dim3(256), 0, s, d_in, ustart_, lens_, slots_, csize_, ovf_, crc_,
                         offs_, out_, (uint32_t)b0);
      DCHK(hipGetLastError());
    }
  }
  offs[nb] = o;
  static const uint8_t kEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                   2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (eof) DCHK(hipMemcpyAsync(out_ + o, kEof, 28, hipMemcpyHostToDevice, s));
  DCHK(hipEventRecord(e1, s));
  DCHK(hipEventSynchronize(e1));
  float t = 0;
  DCHK(hipEventElapsedTime(&t, e0, e1));
  if (ms) *ms = t;
  out_len_ = o + (eof ? 28 : 0);  // only once the output is complete
  for (uint8_t v : ov) fallbacks_ += v;
  return 0;
}

}  // namespace hbam
