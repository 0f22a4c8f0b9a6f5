// hbam_guess.hip -- BAMSplitGuesser on the GPU, all split points in one launch,
// plus a parallel per-block CRC-32 check (the guesser runs
// BlockCompressedInputStream with setCheckCrcs(true), BAMSplitGuesser.java:143).
//
//   k_block_crc     one 256-thread workgroup per BGZF block: per-thread raw
//                   CRC-32 of a slice (LDS table), slices combined with GF(2)
//                   shift operators (x^(8n) mod P) -- zlib crc32_combine math.
//   k_guess_splits  one thread per split point: BaseSplitGuesser.guessNextBGZFPos
//                   over the compressed window, BAMSplitGuesser.guessNextBAMPos over
//                   the GPU-inflated block, then the 3-block decode verification
//                   (BAMSplitGuesser.java:108-339) restated over the inflated stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hbam_device.h"
#include "hbam_host.h"

namespace hbam {

constexpr uint32_t kCrcPoly = 0xedb88320u;

__device__ __host__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
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

// x^(8 n) mod P, reflected (zlib x2nmodp(n, 3))
__device__ inline uint32_t xpow8n(uint64_t n) {
  uint32_t p = 1u << 31;  // x^0
  uint32_t x2n = 1u << 30;  // x^1
  // x^(2^k) table built on the fly: start at k = 3 (x^8)
  for (int k = 0; k < 3; ++k) x2n = multmodp(x2n, x2n);
  while (n) {
    if (n & 1) p = multmodp(x2n, p);
    n >>= 1;
    x2n = multmodp(x2n, x2n);
  }
  return p;
}

__global__ __launch_bounds__(256) void k_block_crc(const BlockInfo* __restrict__ blocks,
                                                   const uint32_t* __restrict__ list, uint32_t nlist,
                                                   const uint8_t* __restrict__ u, uint8_t* __restrict__ ok) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t part[256];
  const uint32_t bi = list[blockIdx.x];
  const BlockInfo b = blocks[bi];
  {
    uint32_t c = threadIdx.x;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    tab[threadIdx.x] = c;
  }
  __syncthreads();
  const uint32_t slice = (b.isize + 255) / 256;
  const uint32_t s0 = min(b.isize, threadIdx.x * slice), s1 = min(b.isize, s0 + slice);
  uint32_t r = 0;  // raw CRC from state 0
  for (uint32_t i = s0; i < s1; ++i) r = tab[(r ^ u[b.ustart + i]) & 0xff] ^ (r >> 8);
  part[threadIdx.x] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t xs = xpow8n(slice);
    uint32_t R = 0xffffffffu;
    for (uint32_t t = 0; t < 256; ++t) {
      const uint32_t a = min(b.isize, t * slice), e = min(b.isize, a + slice);
      if (e == a) continue;
      const uint32_t xp = (e - a == slice) ? xs : xpow8n(e - a);
      R = multmodp(xp, R) ^ part[t];
    }
    ok[bi] = ((R ^ 0xffffffffu) == b.crc) ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
// guesser
// ---------------------------------------------------------------------------
struct GuessEnv {
  const uint8_t* file;     // absolute coordinates
  uint64_t flen;
  const BlockInfo* blocks;
  uint32_t nblk;
  const uint8_t* u;
  const uint8_t* valid;    // per block: inflated OK and CRC OK
  int32_t n_ref;
};

__device__ __forceinline__ uint32_t g_rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t g_rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

// BaseSplitGuesser.guessNextBGZFPos (:31-108) over a[0, alen)
__device__ bool guess_bgzf_pos(const uint8_t* a, uint64_t alen, int32_t p, int32_t end, int32_t* pos, int32_t* size) {
#define NEED(at, k) \
  if ((int64_t)(at) < 0 || (uint64_t)(at) + (k) > alen) return false
  for (;;) {
    for (;;) {
      NEED(p, 4);
      const uint32_t nn = g_rd32(a + p);
      if (nn == 0x04088b1fu) break;
      if ((nn >> 8) == 0x00088b1fu) ++p;
      else if ((nn >> 16) == 0x00008b1fu) p += 2;
      else p += 3;
      if (p >= end) return false;
    }
    const int32_t p0 = p;
    p += 10;
    NEED(p, 2);
    const int32_t xlen = (int32_t)g_rd16(a + p);
    p += 2;
    const int32_t subEnd = p + xlen;
    while (p < subEnd) {
      NEED(p, 4);
      if (g_rd32(a + p) != 0x00024342u) {
        p += 4 + (int32_t)g_rd16(a + p + 2);
        continue;
      }
      NEED(p + 4, 2);
      const int32_t bsize = (int32_t)g_rd16(a + p + 4);
      p += 6;
      while (p < subEnd) {
        NEED(p, 4);
        p += 4 + (int32_t)g_rd16(a + p + 2);
      }
      if (p != subEnd) break;
      p += bsize - xlen - 19 + 4;
      NEED(p, 4);
      *pos = p0;
      *size = (int32_t)g_rd32(a + p);
      return true;
    }
    p = p0 + 4;
  }
#undef NEED
}

__device__ int64_t find_block(const GuessEnv& E, uint64_t coff) {
  uint32_t lo = 0, hi = E.nblk;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (E.blocks[mid].coff < coff) lo = mid + 1; else hi = mid;
  }
  return (lo < E.nblk && E.blocks[lo].coff == coff) ? (int64_t)lo : -1;
}

enum { GZ_OK = 0, GZ_EOF = 1, GZ_TRUNC = 2, GZ_RTIO = 3, GZ_FMT = 4 };

// [htsjdk] BlockCompressedInputStream over the guesser's window, positioned in
// block kb at offset off.
struct GzDev {
  uint32_t kb;
  uint32_t off;
  bool has;      // a current block is loaded
  uint64_t W;    // window end (absolute)
};

__device__ int gz_read_block(const GuessEnv& E, GzDev& g, uint32_t next) {
  if (next >= E.nblk) { g.has = false; return GZ_EOF; }
  const BlockInfo b = E.blocks[next];
  if (b.coff >= g.W) { g.has = false; return GZ_EOF; }
  if (g.W - b.coff < 18) return GZ_RTIO;           // "Incorrect header size" -> RuntimeIOException
  if (b.coff + b.csize > g.W) return GZ_TRUNC;     // FileTruncatedException
  if (!E.valid[next]) return GZ_FMT;               // CRC mismatch / bad DEFLATE
  g.kb = next;
  g.off = 0;
  g.has = true;
  return GZ_OK;
}

// one read(byte[],0,n) call: returns bytes read (0 = EOF / -1 in Java) or -err
__device__ int64_t gz_read_call(const GuessEnv& E, GzDev& g, uint64_t n) {
  uint64_t got = 0;
  while (got < n) {
    if (!g.has) break;
    const uint32_t isz = E.blocks[g.kb].isize;
    if (g.off == isz) {
      int rc = gz_read_block(E, g, g.kb + 1);
      if (rc == GZ_EOF) break;
      if (rc != GZ_OK) return -(int64_t)rc;
      if (E.blocks[g.kb].isize == 0) break;
      continue;
    }
    const uint64_t k = min((uint64_t)(isz - g.off), n - got);
    g.off += (uint32_t)k;
    got += k;
  }
  return (int64_t)got;
}

// BinaryCodec.readBytes / IOUtils.readFully: loop of read calls
__device__ int64_t gz_read_loop(const GuessEnv& E, GzDev& g, uint64_t n) {
  uint64_t got = 0;
  while (got < n) {
    const int64_t r = gz_read_call(E, g, n - got);
    if (r < 0) return r;
    if (r == 0) break;
    got += (uint64_t)r;
  }
  return (int64_t)got;
}

__device__ uint64_t gz_pos(const GuessEnv& E, const GzDev& g) { return E.blocks[g.kb].ustart + g.off; }
__device__ uint64_t gz_tell_coff(const GuessEnv& E, const GzDev& g) {
  const BlockInfo b = E.blocks[g.kb];
  return g.off == b.isize ? b.coff + b.csize : b.coff;
}

__device__ bool valid_aux_dev(const uint8_t* t, int64_t len) {
  int64_t i = 0;
  while (i < len) {
    if (len - i < 3) return false;
    const uint8_t ty = t[i + 2];
    i += 3;
    int64_t sz;
    switch (ty) {
      case 'A': case 'c': case 'C': sz = 1; break;
      case 's': case 'S': sz = 2; break;
      case 'i': case 'I': case 'f': sz = 4; break;
      case 'Z': case 'H': {
        int64_t j = i;
        while (j < len && t[j]) ++j;
        if (j >= len) return false;
        sz = j - i + 1;
        break;
      }
      case 'B': {
        if (len - i < 5) return false;
        const uint8_t sub = t[i];
        const int32_t cnt = (int32_t)g_rd32(t + i + 1);
        int es;
        switch (sub) {
          case 'c': case 'C': es = 1; break;
          case 's': case 'S': es = 2; break;
          case 'i': case 'I': case 'f': es = 4; break;
          default: return false;
        }
        if (cnt < 0) return false;
        sz = 5 + (int64_t)cnt * es;
        break;
      }
      default: return false;
    }
    if (len - i < sz) return false;
    i += sz;
  }
  return true;
}

enum { DEC_OK = 0, DEC_NULL = 1, DEC_REJECT = 2, DEC_TRUNC = 3, DEC_EOF = 4 };

// [htsjdk] BAMRecordCodec.decode + setHeaderStrict + eagerDecode, structurally.
__device__ int decode_verify(const GuessEnv& E, GzDev& g) {
  const uint64_t q = gz_pos(E, g);
  int64_t r = gz_read_loop(E, g, 4);
  if (r < 0) return r == -GZ_TRUNC ? DEC_TRUNC : DEC_REJECT;
  if (r < 4) return DEC_NULL;
  // the 4 bytes may lie after skipped empty blocks: they are contiguous in u
  const int32_t bs = (int32_t)g_rd32(E.u + q);
  if (bs < 32) return DEC_REJECT;
  r = gz_read_loop(E, g, (uint64_t)bs);
  if (r < 0) return r == -GZ_TRUNC ? DEC_TRUNC : DEC_REJECT;
  if (r < bs) return DEC_EOF;
  const uint8_t* rec = E.u + q + 4;
  const int32_t ref = (int32_t)g_rd32(rec), nref = (int32_t)g_rd32(rec + 20);
  if (ref < -1 || ref >= E.n_ref || nref < -1 || nref >= E.n_ref) return DEC_REJECT;
  const int32_t lrn = rec[8], ncig = (int32_t)g_rd16(rec + 12), lseq = (int32_t)g_rd32(rec + 16);
  const int64_t rest = bs - 32;
  const uint8_t* v = rec + 32;
  if (lrn < 1 || lrn - 1 > rest) return DEC_REJECT;
  if ((int64_t)lrn + 4 * (int64_t)ncig > rest) return DEC_REJECT;
  for (int32_t k = 0; k < ncig; ++k)
    if ((g_rd32(v + lrn + 4 * k) & 0xf) > 8) return DEC_REJECT;
  const int64_t seqoff = (int64_t)lrn + 4 * (int64_t)ncig;
  if (lseq < 0) return DEC_REJECT;
  if (lseq > 0 && seqoff + ((int64_t)lseq + 1) / 2 > rest) return DEC_REJECT;
  const int64_t tagoff = seqoff + ((int64_t)lseq + 1) / 2 + lseq;
  if (tagoff > rest) return DEC_REJECT;
  if (!valid_aux_dev(v + tagoff, rest - tagoff)) return DEC_REJECT;
  return DEC_OK;
}

// guessNextBAMPos (:237-339) within block k (all reads stay inside the block)
__device__ int32_t guess_bam_pos(const GuessEnv& E, uint32_t k, int32_t up, int32_t cSize) {
  const uint8_t* d = E.u + E.blocks[k].ustart;
  up += 4;
  for (;;) {
    if (!(up + 35 < cSize)) return -1;
    const int32_t id = (int32_t)g_rd32(d + up), pos = (int32_t)g_rd32(d + up + 4);
    if (id < -1 || id > E.n_ref || pos < -1) { ++up; continue; }
    const int32_t nid = (int32_t)g_rd32(d + up + 20), npos = (int32_t)g_rd32(d + up + 24);
    if (nid < -1 || nid > E.n_ref || npos < -1) { ++up; continue; }
    const int32_t nextUP = up + 1;
    up -= 4;
    const int32_t nameLength = (int32_t)(g_rd32(d + up + 12) & 0xff);
    if (nameLength < 1) { up = nextUP; continue; }
    const int32_t nullTerminator = up + 36 + nameLength - 1;
    if (nullTerminator >= cSize) { up = nextUP; continue; }
    if (d[nullTerminator] != 0) { up = nextUP; continue; }
    int32_t zeroMin = 4 * 8 + nameLength;
    zeroMin = (int32_t)((uint32_t)zeroMin + (uint32_t)(((int32_t)g_rd32(d + up + 16) & 0xffff) * 4));
    const int32_t l20 = (int32_t)g_rd32(d + up + 20);
    zeroMin = (int32_t)((uint32_t)zeroMin + (uint32_t)l20 + (uint32_t)((int32_t)((uint32_t)l20 + 1u) / 2));
    if ((int32_t)g_rd32(d + up) < zeroMin) { up = nextUP; continue; }
    return up;
  }
}

constexpr uint64_t kMaxBytesRead = 3 * 0xffff + 0xfffe;  // :66-73

__global__ void k_guess_splits(GuessEnv E, const uint64_t* __restrict__ begs, const uint64_t* __restrict__ ends,
                               uint32_t n, uint64_t* __restrict__ out, int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t beg = begs[i], end = ends[i];
  uint64_t want = min(end - beg, kMaxBytesRead);
  if (beg + want > E.flen) want = E.flen > beg ? E.flen - beg : 0;
  const uint8_t* a = E.file + beg;
  const uint64_t W = beg + want;
  const int32_t firstEnd = (int32_t)min(end - beg, (uint64_t)0xffff);
  status[i] = kOk;
  for (int32_t cp = 0;; ++cp) {
    int32_t ppos, psize;
    if (!guess_bgzf_pos(a, want, cp, firstEnd, &ppos, &psize)) { out[i] = end; return; }
    const int32_t cp0 = cp = ppos;
    // bgzf.seek(cp0 << 16): a real block fully inside the window, inflating with a good CRC
    const int64_t kb = find_block(E, beg + (uint64_t)cp0);
    if (kb < 0) continue;
    const BlockInfo b = E.blocks[kb];
    if (b.coff + b.csize > W || !E.valid[kb] || b.isize == 0) continue;
    for (int32_t up = 0;; ++up) {
      const int32_t up0 = up = guess_bam_pos(E, (uint32_t)kb, up, psize);
      if (up0 < 0) break;
      GzDev g;
      g.kb = (uint32_t)kb;
      g.off = (uint32_t)up0;
      g.has = true;
      g.W = W;
      bool decodedAny = false, accept = true;
      int blocks_seen = 0;
      uint64_t prevCP = b.coff;
      while (blocks_seen < 3) {
        const int dr = decode_verify(E, g);
        if (dr == DEC_NULL) break;
        if (dr == DEC_REJECT) { accept = false; break; }
        if (dr == DEC_TRUNC || dr == DEC_EOF) {  // in.eof() holds once the reader hit the window end
          if (!decodedAny) accept = false;
          break;
        }
        decodedAny = true;
        const uint64_t cp2 = gz_tell_coff(E, g);
        if (cp2 != prevCP) { prevCP = cp2; ++blocks_seen; }
      }
      if (accept && blocks_seen < 3 && !decodedAny) accept = false;
      if (!accept) continue;
      out[i] = ((beg + (uint64_t)cp0) << 16) | (uint64_t)up0;
      return;
    }
  }
}

// util/BGZFSplitGuesser.java:64-167 (guessNextBGZFBlockStart): its own
// guessNextBGZFPos over arr = file[beg, beg + min(end-beg, 2*0xffff-1)),
// candidates below firstBGZFEnd = min(end-beg, 0xffff); the first candidate
// whose block reads whole from arr and inflates with a good CRC wins.
// in.read past the array end keeps the stale bytes of buf
// (ByteArraySeekableStream), restated with a per-lane 4-byte buffer.
constexpr uint64_t kBgzfGuessWindow = 2 * 0xffff - 1;  // :74

__global__ void k_guess_bgzf_starts(GuessEnv E, const uint64_t* __restrict__ begs, const uint64_t* __restrict__ ends,
                                    uint32_t n, uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t beg = begs[i], end = ends[i];
  uint64_t alen = min(end - beg, kBgzfGuessWindow);
  if (beg + alen > E.flen) alen = E.flen > beg ? E.flen - beg : 0;
  const uint8_t* a = E.file + beg;
  const int32_t firstEnd = (int32_t)min(end - beg, (uint64_t)0xffff);
  uint8_t buf[4] = {0, 0, 0, 0};
  for (int32_t pos = 0;;) {
    int32_t p = pos, got = -1;
    for (;;) {  // guessNextBGZFPos (:114-166)
      bool stop = false;
      for (;;) {
        for (int k = 0; k < 4; ++k) {  // in.seek(p); in.read(buf, 0, 4)
          if (p >= 0 && (uint64_t)p + k < alen) buf[k] = a[p + k];
          else if (k == 0 && (uint64_t)p >= alen) break;
        }
        const uint32_t nn = g_rd32(buf);
        if (nn == 0x04088b1fu) break;
        if ((nn >> 8) == (0x04088b1fu & 0xffffffu)) ++p;
        else if ((nn >> 16) == (0x04088b1fu & 0xffffu)) p += 2;
        else p += 3;
        if (p >= firstEnd) { stop = true; break; }
      }
      if (stop) break;
      const int32_t p0 = p;
      p += 12;
      if ((uint64_t)p0 + 12 > alen) break;
      const int32_t xlen = (int32_t)g_rd16(a + p0 + 10), subEnd = p + xlen;
      while (p < subEnd) {
        if ((uint64_t)p + 4 > alen) break;
        if (g_rd32(a + p) != 0x00024342u) { p += 4 + (int32_t)g_rd16(a + p + 2); continue; }
        got = p0;
        break;
      }
      if (got >= 0) break;
      p = p0 + 4;
    }
    if (got < 0) { out[i] = end; return; }
    pos = got;
    // bgzf.seek(pos << 16): a real block read whole from arr, inflating with a good CRC
    const int64_t kb = find_block(E, beg + (uint64_t)pos);
    if (kb >= 0) {
      const BlockInfo b = E.blocks[kb];
      if (b.coff + b.csize <= beg + alen && E.valid[kb] && (b.isize > 0 || b.crc == 0)) {
        out[i] = beg + (uint64_t)pos;
        return;
      }
    }
    ++pos;
  }
}

}  // namespace hbam

// ---------------------------------------------------------------------------
// host drivers: hadoop_bam::guess_batch / guess_bgzf_batch
// ---------------------------------------------------------------------------
// Each split point reads at most a few hundred KB after its start
// (BAMSplitGuesser.java:127-138 MAX_BYTES_READ; BGZFSplitGuesser.java:74), so
// the points are grouped into windows of nearby ranges; a window is loaded
// from its first point's offset (free start: the block chain begins at the
// first header candidate whose BSIZE chain runs through the window, a byte
// offset need not be a block start), every block in it is inflated and CRC
// checked, and one launch guesses all of its points.  One extra 64 KiB keeps
// a block that straddles a point's read limit in the table, so the limit
// checks see it exactly as over the whole file.
namespace hadoop_bam {

namespace {
struct GuessPoint {
  uint64_t beg, end, lim;  // lim: end of the bytes the guesser may read
  size_t slot;
};

// Windows over sorted points: [lo, hi) covering points [a, b).
template <typename F>
int for_each_window(BamFile& f, std::vector<GuessPoint>& pts, F&& body) {
  std::sort(pts.begin(), pts.end(), [](const GuessPoint& x, const GuessPoint& y) { return x.beg < y.beg; });
  const uint64_t size = f.file_size(), cap = std::max<uint64_t>(f.window_bytes(), 1ull << 20);
  for (size_t a = 0; a < pts.size();) {
    const uint64_t lo = pts[a].beg;
    uint64_t hi = std::min(size, pts[a].lim + 0x10000);
    size_t b = a + 1;
    while (b < pts.size() && pts[b].beg <= hi + (1ull << 20)) {
      const uint64_t h2 = std::max(hi, std::min(size, pts[b].lim + 0x10000));
      if (h2 - lo > cap) break;
      hi = h2;
      ++b;
    }
    int rc = body(lo, hi, a, b);
    if (rc != hbam::kOk) return rc;
    a = b;
  }
  return hbam::kOk;
}

// Load + locate + inflate + CRC-check the window; *valid[k] per block.
int prepare_window(BamFile& f, uint64_t lo, uint64_t hi, hbam::DevBuf<uint8_t>* dvalid, std::string* err) {
  using namespace hbam;
  int rc = f.load_window(lo, hi, /*free_start=*/true);
  if (rc != kOk) {
    *err = f.error();
    return rc;
  }
  Pipeline& p = f.pipe();
  const auto& blk = p.blocks();
  const uint32_t nblk = (uint32_t)blk.size();
  std::vector<uint8_t> valid(nblk, 0);
  std::vector<uint32_t> dev_idx;
  if (nblk) {
    // inflate errors mark blocks invalid, as a failed seek would
    if (p.inflate(0, nblk) == kOk) {
      for (uint32_t j = 0; j < nblk; ++j) valid[j] = 1;
    } else {
      for (uint32_t j = 0; j < nblk; ++j) valid[j] = p.inflate(j, j + 1) == kOk;
    }
    for (uint32_t j = 0; j < nblk; ++j)
      if (valid[j] && blk[j].isize > 0) dev_idx.push_back(j);
  }
  DevBuf<uint32_t> dlist(&p.streams());
  hipStream_t s = p.stream();
  auto chk = [&](hipError_t e) {
    if (e != hipSuccess) *err = std::string("HIP: ") + hipGetErrorString(e);
    return e == hipSuccess;
  };
  if (!chk(dvalid->reserve(nblk + 1)) || !chk(dlist.reserve(dev_idx.size() + 1))) return kErrDevice;
  if (nblk && !chk(hipMemcpyAsync(dvalid->p, valid.data(), nblk, hipMemcpyHostToDevice, s))) return kErrDevice;
  if (!dev_idx.empty()) {  // setCheckCrcs(true): valid[k] = CRC ok
    if (!chk(hipMemcpyAsync(dlist.p, dev_idx.data(), dev_idx.size() * 4, hipMemcpyHostToDevice, s))) return kErrDevice;
    hipLaunchKernelGGL(k_block_crc, dim3((uint32_t)dev_idx.size()), dim3(256), 0, s, p.d_blocks(), dlist.p,
                       (uint32_t)dev_idx.size(), p.d_u(), dvalid->p);
    if (!chk(hipGetLastError())) return kErrDevice;
  }
  if (!chk(hipStreamSynchronize(s))) return kErrDevice;
  return kOk;
}

// points [a, b) through kernel K; results into out by slot
template <typename Launch>
int run_points(BamFile& f, const std::vector<GuessPoint>& pts, size_t a, size_t b, const hbam::DevBuf<uint8_t>& dvalid,
               std::vector<uint64_t>* out, std::string* err, int32_t n_ref, Launch&& launch) {
  using namespace hbam;
  Pipeline& p = f.pipe();
  const uint32_t m = (uint32_t)(b - a);
  std::vector<uint64_t> hb(m), he(m), res(m);
  for (uint32_t j = 0; j < m; ++j) {
    hb[j] = pts[a + j].beg;
    he[j] = pts[a + j].end;
  }
  DevBuf<uint64_t> dbeg(&p.streams()), dend(&p.streams()), dout(&p.streams());
  DevBuf<int32_t> dst(&p.streams());
  hipStream_t s = p.stream();
  auto chk = [&](hipError_t e) {
    if (e != hipSuccess) *err = std::string("HIP: ") + hipGetErrorString(e);
    return e == hipSuccess;
  };
  if (!chk(dbeg.reserve(m)) || !chk(dend.reserve(m)) || !chk(dout.reserve(m)) || !chk(dst.reserve(m)))
    return kErrDevice;
  if (!chk(hipMemcpyAsync(dbeg.p, hb.data(), m * 8, hipMemcpyHostToDevice, s)) ||
      !chk(hipMemcpyAsync(dend.p, he.data(), m * 8, hipMemcpyHostToDevice, s)))
    return kErrDevice;
  GuessEnv E;
  E.file = p.d_file() - p.base();  // absolute file coordinates (the window covers every point's bytes)
  E.flen = f.file_size();
  E.blocks = p.d_blocks();
  E.nblk = (uint32_t)p.blocks().size();
  E.u = p.d_u();
  E.valid = dvalid.p;
  E.n_ref = n_ref;
  launch(E, dbeg.p, dend.p, m, dout.p, dst.p, s);
  if (!chk(hipGetLastError())) return kErrDevice;
  if (!chk(hipMemcpyAsync(res.data(), dout.p, m * 8, hipMemcpyDeviceToHost, s)) || !chk(hipStreamSynchronize(s)))
    return kErrDevice;
  for (uint32_t j = 0; j < m; ++j) (*out)[pts[a + j].slot] = res[j];
  return kOk;
}
}  // namespace

int guess_batch(BamFile& f, const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                std::vector<uint64_t>* out, std::string* err, int32_t n_ref) {
  using namespace hbam;
  const size_t n = begs.size();
  out->assign(n, 0);
  std::vector<GuessPoint> pts;
  for (size_t i = 0; i < n; ++i) {
    if (ends[i] < begs[i]) {
      *err = "split end before its start";
      return kErrArg;
    }
    if (begs[i] == 0) {  // :115-123 the header gives the first record
      (*out)[i] = f.first_record_voff();
      continue;
    }
    if (begs[i] >= f.file_size()) {  // nothing to read: no record start
      (*out)[i] = ends[i];
      continue;
    }
    const uint64_t lim = std::min<uint64_t>(begs[i] + std::min<uint64_t>(ends[i] - begs[i], kMaxBytesRead), f.file_size());
    pts.push_back({begs[i], ends[i], lim, i});
  }
  DevBuf<uint8_t> dvalid(&f.pipe().streams());
  return for_each_window(f, pts, [&](uint64_t lo, uint64_t hi, size_t a, size_t b) {
    int rc = prepare_window(f, lo, hi, &dvalid, err);
    if (rc != kOk) return rc;
    return run_points(f, pts, a, b, dvalid, out, err, n_ref < 0 ? f.n_ref() : n_ref,
                      [](const GuessEnv& E, const uint64_t* db, const uint64_t* de, uint32_t m, uint64_t* dout,
                         int32_t* dst, hipStream_t s) {
                        hipLaunchKernelGGL(k_guess_splits, dim3((m + 63) / 64), dim3(64), 0, s, E, db, de, m, dout,
                                           dst);
                      });
  });
}

int guess_bgzf_batch(BamFile& f, const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                     std::vector<uint64_t>* out, std::string* err) {
  using namespace hbam;
  const size_t n = begs.size();
  out->assign(n, 0);
  std::vector<GuessPoint> pts;
  for (size_t i = 0; i < n; ++i) {
    if (ends[i] < begs[i]) {
      *err = "split end before its start";
      return kErrArg;
    }
    if (begs[i] >= f.file_size()) {
      (*out)[i] = ends[i];
      continue;
    }
    const uint64_t lim =
        std::min<uint64_t>(begs[i] + std::min<uint64_t>(ends[i] - begs[i], kBgzfGuessWindow), f.file_size());
    pts.push_back({begs[i], ends[i], lim, i});
  }
  DevBuf<uint8_t> dvalid(&f.pipe().streams());
  return for_each_window(f, pts, [&](uint64_t lo, uint64_t hi, size_t a, size_t b) {
    int rc = prepare_window(f, lo, hi, &dvalid, err);
    if (rc != kOk) return rc;
    return run_points(f, pts, a, b, dvalid, out, err, f.n_ref(),
                      [](const GuessEnv& E, const uint64_t* db, const uint64_t* de, uint32_t m, uint64_t* dout,
                         int32_t*, hipStream_t s) {
                        hipLaunchKernelGGL(k_guess_bgzf_starts, dim3((m + 63) / 64), dim3(64), 0, s, E, db, de, m,
                                           dout);
                      });
  });
}

}  // namespace hadoop_bam
