// hbam_kernels.hip -- gfx950 kernels for the Hadoop-BAM read hot path.
//
//   bgzf_scan -> sort -> bgzf_verify (bgzf_walk fallback)   BGZF block discovery
//        ([htsjdk] BlockCompressedInputStream.readBlock; heuristic twin
//         BaseSplitGuesser.java:31-108)
//   huff_tables    one wave per block: a DEFLATE block's header + Huffman
//        tables, built ahead of the decode at high occupancy (in rounds: the
//        first block of each BGZF block, then the one the decode stopped at)
//   inflate_huff   (phase A) one 256-thread workgroup per BGZF block: the
//        symbol stream -> LZ77 tokens by 256 speculative slices, a sync pass
//        and an emit pass; the compressed block and the tables sit in LDS.
//        ([htsjdk] BlockGunzipper.unzipBlock -> java.util.zip.Inflater)
//   inflate_lz77   (phase B) one 1024-thread workgroup per BGZF block: tokens
//        -> a u16 LDS map (literal or source position), resolved by pointer
//        chasing with path compression, 16 B coalesced stores into the
//        contiguous inflated stream.
//   rec_cand / rec_walk / rec_search / rec_linkfix / rec_check   BAM
//        record-boundary chain ([htsjdk] BAMRecordCodec.decode;
//        SplittingBAMIndexer.java:340-368) with the STRICT isValid rules
//   rec_out        fused field decode + sort key + voff
//        (LazyBAMRecordFactory.java:37-50; BAMRecordReader.java:81-121;
//         util/MurmurHash3.java:32-102); long_hash for rests > 2 KiB
//   sbi_emit       .splitting-bai entries (SplittingBAMIndexer.java:262-287)
//   wr_copy / wr_bin_patch / wr_decode   SAMRecordWritable.write / readFields
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stddef.h>
#include <stdint.h>

#include "hbam_device.h"
#include "hbam_launch.h"

namespace hbam {

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// unaligned little-endian u32 from a 4-aligned base (reads 8 bytes: pad!)
__device__ __forceinline__ uint32_t ldu32(const uint8_t* base, uint64_t off) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (off & ~3ull));
  uint32_t lo = p[0], hi = p[1];
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ uint64_t ldu64(const uint8_t* base, uint64_t off) {
  return (uint64_t)ldu32(base, off) | ((uint64_t)ldu32(base, off + 4) << 32);
}

// A record's block_size and 32 fixed-field bytes (q .. q + 36) from three
// dword-aligned loads (two dwordx4, one dwordx2) instead of one ldu32 (two
// dword loads) per field: the record walks and the check/output pass issue
// ~6x fewer load instructions per record.  at(k) = the u32 at q + 4k, k <= 8.
// Reads up to 3 bytes past q + 36 (the stream is padded).
struct __attribute__((aligned(4))) U32x4 { uint32_t x, y, z, w; };
struct __attribute__((aligned(4))) U32x2 { uint32_t x, y; };
struct RecHead {
  uint32_t w[10];
  uint32_t sh;
  __device__ __forceinline__ uint32_t at(int k) const { return __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh); }
};
__device__ __forceinline__ RecHead load_head(const uint8_t* base, uint64_t q) {
  const uint8_t* b = base + (q & ~3ull);
  const U32x4 a = *reinterpret_cast<const U32x4*>(b);
  const U32x4 c = *reinterpret_cast<const U32x4*>(b + 16);
  const U32x2 d = *reinterpret_cast<const U32x2*>(b + 32);
  RecHead h;
  h.w[0] = a.x; h.w[1] = a.y; h.w[2] = a.z; h.w[3] = a.w;
  h.w[4] = c.x; h.w[5] = c.y; h.w[6] = c.z; h.w[7] = c.w;
  h.w[8] = d.x; h.w[9] = d.y;
  h.sh = (uint32_t)(q & 3);
  return h;
}

// ---------------------------------------------------------------------------
// BGZF block discovery
// ---------------------------------------------------------------------------
// A candidate is a position whose 16 header bytes read 1f 8b 08 04 .. .. .. ..
// .. .. 06 00 'B' 'C' 02 00 (ID1 ID2 CM FLG, XLEN=6, BC subfield, SLEN=2): the
// exact framing htsjdk writes and requires (XLEN==6), plus the BC subfield id
// for selectivity.  Candidates are appended unordered, sorted, then the BSIZE
// chain is verified; any break falls back to the serial walk (bgzf_walk).
__global__ __launch_bounds__(256) void k_bgzf_scan(const uint8_t* __restrict__ buf, uint64_t len, uint64_t base,
                                                   uint64_t from, uint64_t* __restrict__ cand, uint32_t cap,
                                                   uint32_t* __restrict__ count) {
  // buf = first byte of the loaded range (16 B aligned, zero padded past
  // len).  Lane i of a wave step reads 16 B chunk c = step + i: one coalesced
  // 1 KiB load per wave (64 B per lane, as before, strided the wave's loads
  // 64 B apart and ran at 2.2 TB/s).  The 4 bytes after a chunk, which a
  // header starting in its last 3 bytes needs, come from the next lane's
  // chunk (a lane shuffle; the wave's last lane loads them).  A word without
  // a 0x1f byte (nearly all of them) costs three VALU operations; the rare
  // 0x1f bytes get the full header test.  Candidates are reported in file
  // coordinates (base + offset).
  // Four such wave steps per iteration (4 KiB per wave), their loads issued
  // together: one load in flight per wave left the scan latency-bound.  The
  // last lane's 4 bytes past the iteration's last chunk are loaded with them
  // (loaded at their use, they cost a second memory latency per iteration).
#ifndef HBAM_SCAN_U
#define HBAM_SCAN_U 4
#endif
#ifndef HBAM_SCAN_PIPE
#define HBAM_SCAN_PIPE 1
#endif
#ifndef HBAM_SCAN_GRID
#define HBAM_SCAN_GRID 8192
#endif
  constexpr int kU = HBAM_SCAN_U;
  // Candidates are collected per workgroup in LDS and reserved in cand[] by
  // one global atomic per workgroup: every candidate's own atomicAdd on one
  // device-scope counter serialized across the 8 XCDs.
  constexpr uint32_t kWgCand = 256;
  __shared__ uint64_t s_cand[kWgCand];
  __shared__ uint32_t s_n, s_base;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint64_t nc = (len + 15) / 16;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kU;
  const uint32_t lane = lane_id();
  const uint64_t wave0 = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * kU;
  // the iteration's kU chunks per lane and the last lane's 4 bytes past them
  // (buf is zero padded past len)
  auto fetch = [&](uint64_t c0, uint4* vv, uint32_t& tail) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t c = c0 + 64 * u + lane;
      vv[u] = c < nc ? reinterpret_cast<const uint4*>(buf)[c] : make_uint4(0, 0, 0, 0);
    }
    const uint64_t clast = c0 + 64 * (kU - 1) + 63;
    tail = lane == 63 && clast < nc ? *reinterpret_cast<const uint32_t*>(buf + 16 * clast + 16) : 0u;
  };
#if HBAM_SCAN_PIPE
  // software-pipelined: the next iteration's loads are in flight while this
  // one's chunks are tested
  uint4 nv[kU];
  uint32_t ntail = 0;
  if (wave0 < nc) fetch(wave0, nv, ntail);
#endif
  for (uint64_t c0 = wave0; c0 < nc; c0 += stride) {
    uint4 vv[kU];
    uint32_t tail;
#if HBAM_SCAN_PIPE
#pragma unroll
    for (int u = 0; u < kU; ++u) vv[u] = nv[u];
    tail = ntail;
    if (c0 + stride < nc) fetch(c0 + stride, nv, ntail);
#else
    fetch(c0, vv, tail);
#endif
#pragma unroll
    for (int u = 0; u < kU; ++u) {
    const uint64_t c = c0 + 64 * u + lane;  // the wave stays converged through the shuffle
    const uint4 v = vv[u];
    uint32_t nx = (uint32_t)__shfl_down((int)v.x, 1, 64);
    // the wave's last lane: the next step's first chunk (lane 0), or the tail
    const uint32_t next0 = u + 1 < kU ? (uint32_t)__shfl((int)vv[u + 1 < kU ? u + 1 : u].x, 0, 64) : 0u;
    if (lane == 63) nx = u + 1 < kU ? next0 : tail;
    const uint32_t w[5] = {v.x, v.y, v.z, v.w, nx};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = w[k] ^ 0x1f1f1f1fu;
      uint32_t hz = (x - 0x01010101u) & ~x & 0x80808080u;  // a byte of w[k] may be 0x1f (superset)
      while (hz) {
        const uint32_t byte = (uint32_t)__builtin_ctz(hz) >> 3;
        hz &= hz - 1;
        const uint32_t magic = __builtin_amdgcn_alignbyte(w[k + 1], w[k], byte);
        if (magic != 0x04088b1fu) continue;
        const uint64_t p = 16 * c + 4 * k + byte;
        if (p + 18 > len || base + p < from) continue;
        const uint32_t xlen = ldu32(buf, p + 10) & 0xffffu;
        const uint32_t sub = ldu32(buf, p + 12);
        if (xlen != 6 || sub != 0x00024342u) continue;
        const uint32_t j = atomicAdd(&s_n, 1u);
        if (j < kWgCand) {
          s_cand[j] = base + p;
        } else {  // (more than kWgCand block headers in one workgroup's range: tiny blocks)
          const uint32_t i = atomicAdd(count, 1u);
          if (i < cap) cand[i] = base + p;
        }
      }
    }
    }
  }
  __syncthreads();
  const uint32_t nw = min(s_n, kWgCand);
  if (threadIdx.x == 0) s_base = nw ? atomicAdd(count, nw) : 0u;
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nw; t += blockDim.x)
    if (s_base + t < cap) cand[s_base + t] = s_cand[t];
}

// Verify the sorted candidate chain and fill BlockInfo.  flags[0] |= 1 on any
// break (fallback), flags[1] = first block index with ISIZE > 64 KiB,
// flags[3] += the empty blocks (ISIZE 0: candidates for dead positions).
// partial (streamed upload, bytes past hi not there yet): a last candidate
// whose block runs past hi is the incomplete tail -> flags[2] = 1, not a break.
__global__ void k_bgzf_verify(const uint8_t* __restrict__ file, uint64_t lo, uint64_t hi,
                              const uint64_t* __restrict__ cand, uint32_t n,
                              BlockInfo* __restrict__ blocks, uint32_t* __restrict__ flags, uint32_t partial) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t c = cand[i];
  if (i == 0 && c != lo) atomicOr(&flags[0], 1u);
  uint32_t total = (ldu32(file, c + 16) & 0xffffu) + 1;
  uint64_t next = c + total;
  uint64_t expect = (i + 1 < n) ? cand[i + 1] : hi;
  if (partial && i + 1 == n && next > hi && total >= 26) {
    flags[2] = 1u;
    return;
  }
  if (next != expect || total < 26) {
    atomicOr(&flags[0], 1u);
    return;
  }
  BlockInfo b;
  b.coff = c;
  b.ustart = 0;
  b.csize = total;
  b.crc = ldu32(file, next - 8);
  b.isize = ldu32(file, next - 4);
  b.flags = 0;
  if (b.isize > kMaxIsize) atomicMin(&flags[1], i);
  if (b.isize == 0) atomicAdd(&flags[3], 1u);
  blocks[i] = b;
}

// Serial fallback: walk BSIZE from lo with htsjdk's framing rules.
// out[0] = nblocks, out[1] = status, out[2] = failing offset (low 32), out[3] = hi 32.
// partial: a block cut by hi ends the walk cleanly (out[2..3] = its start).
__global__ void k_bgzf_walk(const uint8_t* __restrict__ file, uint64_t lo, uint64_t hi,
                            BlockInfo* __restrict__ blocks, uint32_t cap, uint32_t* __restrict__ out,
                            uint32_t partial) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t p = lo;
  uint32_t n = 0;
  int st = kOk;
  while (p < hi) {
    if (hi - p < 18) { st = partial ? kOk : kErrIO; break; }
    uint32_t total = (ldu32(file, p + 16) & 0xffffu) + 1;
    if (total < 18) { st = kErrIO; break; }
    if (p + total > hi) { st = partial ? kOk : kErrTrunc; break; }
    uint32_t w0 = ldu32(file, p);
    uint32_t xlen = ldu32(file, p + 10) & 0xffffu;
    if (w0 != 0x04088b1fu || xlen != 6 || total < 26) { st = kErrFormat; break; }
    if (n >= cap) { st = kErrState; break; }
    BlockInfo b;
    b.coff = p;
    b.ustart = 0;
    b.csize = total;
    b.crc = ldu32(file, p + total - 8);
    b.isize = ldu32(file, p + total - 4);
    b.flags = 0;
    if (b.isize > kMaxIsize) { st = kErrFormat; break; }
    blocks[n++] = b;
    p += total;
  }
  out[0] = n;
  out[1] = (uint32_t)st;
  out[2] = (uint32_t)p;
  out[3] = (uint32_t)(p >> 32);
}

__global__ void k_block_isize(const BlockInfo* __restrict__ blocks, uint32_t n, uint64_t* __restrict__ isz) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) isz[i] = blocks[i].isize;
}
__global__ void k_block_ustart(BlockInfo* __restrict__ blocks, uint32_t n, const uint64_t* __restrict__ us,
                               uint64_t base) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) blocks[i].ustart = base + us[i];
}

// ---------------------------------------------------------------------------
// Inflate phase A: Huffman decode, one 256-thread workgroup per BGZF block
// ---------------------------------------------------------------------------
// The block's compressed bytes are staged in LDS (dynamic shared memory sized
// per launch to the largest block of the chunk) by coalesced 16 B loads; the
// Huffman tables (~11 KiB) sit next to them.  Wave 0 parses block headers,
// decodes code lengths and builds the tables (wave-uniform scalar code, the
// other waves wait at a barrier).  A DEFLATE block's symbol stream is then
// decoded by all 256 lanes at once: lane l starts at a guessed bit position
// B0 + l*S and decodes its slice up to the first symbol boundary at or past
// the next slice (its "exit").  Huffman streams self-synchronise, so a lane
// that started off a boundary soon falls onto the true path.  A sync pass
// re-decodes each slice from its predecessor's exit only until it lands on one
// of the first kMergePts boundaries its speculative walk recorded (the walks
// share every symbol from there on), so it costs a few symbols per lane.  A
// last pass re-decodes each slice from its true start and writes tokens at
// workgroup-scanned offsets, four at a time (16 B stores).
//
// Semantics follow zlib's inflate() as driven by [htsjdk] BlockGunzipper
// (one call, all input, ISIZE bytes of output space):
//   * a field whose bits are not all inside the block's CDATA stops decoding
//     ("Did not inflate expected amount" = kErrFormat unless output is full);
//   * invalid codes / distances -> DataFormatException (kErrIO);
//   * once output is exactly full at a symbol boundary, zlib still decodes the
//     next litlen code (and a whole length/distance pair, or the next block
//     header after an end-of-block) before it notices there is no room: those
//     can still raise errors -> the scalar lookahead below.
//
// Table entries (u32):
//   litlen  [15:0] payload  [20:16] bits to consume  [25:24] literal count  [28:26] kind
//           kind 0 LIT : payload = 1 or 2 literal bytes; (e & 0x0300ffff) IS the token
//           kind 1 LEN : payload [8:0] base (3..258), [12:9] extra bits
//           kind 2 EOB, 3 LONG (payload = sub-table base), 4 BAD, 5 SLOW (canonical decode)
//   dist    [14:0] base  [20:16] bits  [24:21] extra  [28:26] kind (0 ok, 3 LONG, 4 BAD, 5 SLOW)
//   codes   [15:0] symbol [20:16] bits (code-length alphabet, root 7: always direct)
// Codes longer than the root index a fixed-size sub-table by the next bits;
// sub-table entries carry the full code length.
// Tokens (u32): literal  bit31=0, [25:24] count (1..2), [15:0] bytes
//               match    bit31=1, [30:16] dist-1, [15:0] length
#ifndef HBAM_HUFF_THREADS
#define HBAM_HUFF_THREADS 256
#endif
constexpr int kHuffThreads = HBAM_HUFF_THREADS;  // lanes per DEFLATE block (a multiple of 64)
constexpr int kHuffWaves = kHuffThreads / 64;
// Phase A reads the compressed block from an LDS copy (staged) or straight
// from HBM/L2, per chunk: staged while the workgroup's LDS (tables + the
// chunk's largest block) leaves room for 4 workgroups per CU, else unstaged
// (C4: 7.4 -> 3.9 ms; C2: staged 7.6 vs 8.0 ms).
#ifndef HBAM_HUFF_STAGE_MAX
#define HBAM_HUFF_STAGE_MAX (40 * 1024)
#endif
constexpr uint32_t kHuffStageMaxLds = HBAM_HUFF_STAGE_MAX;

// Wave-local ordering of LDS traffic (code run by one wave only).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int kLitRoot = 10;
constexpr int kDistRoot = 9;
// Variable-size sub-tables (as zlib's inflate_table): the root entry of a
// long-code prefix holds the sub-table base and its index width (= the longest
// code under that prefix - root).  A complete litlen code with a 10-bit root
// needs at most 310 sub entries (zlib ENOUGH_LENS 1334 - 1024), the distance
// code with a 9-bit root at most 80 (ENOUGH_DISTS 592 - 512); build_table
// accepts complete codes only (and the one-code case).  Prefixes that would
// not fit fall back to K_SLOW (canonical decode), which valid streams never
// reach.  The caps size the table image every block writes and phase A reads
// back, and the LDS that bounds k_huff_tables' resident waves.
constexpr int kLitSubCap = 320;
constexpr int kDistSubCap = 128;
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_LONG = 3, K_BAD = 4, K_SLOW = 5 };
constexpr uint32_t kBadEntry = K_BAD << 26;
constexpr uint32_t kLongTag = 0xF0000000u;  // build-time mark: kLongTag | (max len - root)
constexpr uint32_t kKindLit = 1u << 26;  // e < kKindLit  <=>  literal entry
// a root entry that points to a sub-table (kind K_LONG) also carries bit 31,
// so the decode loop tests it with one signed compare
constexpr uint32_t kLongEntry = 0x80000000u | (K_LONG << 26);
__device__ __forceinline__ bool is_long(uint32_t e) { return (int32_t)e < 0; }

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,
                                       33,  49,  65,  97,  129, 193,  257,  385,  513,  769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// LDS tables of one DEFLATE block.  The leading kTableImage bytes (lit ..
// sort_dist) are everything the symbol decode reads; k_huff_tables writes
// exactly that image to HBM and k_inflate_huff copies it back.
struct HuffLds {
  uint32_t lit[1 << kLitRoot];                      // litlen root table (with literal pairs)
  uint32_t litsub[kLitSubCap];                      // litlen sub-tables
  uint32_t dist[1 << kDistRoot];                    // distance root table (also the code-length table)
  uint32_t distsub[kDistSubCap];                    // distance sub-tables
  uint32_t cnt_lit[16];
  uint32_t cnt_dist[16];
  uint16_t sort_lit[288];
  uint16_t sort_dist[32];
  // ---- build scratch
  uint32_t offs[16];
  uint32_t firstc[16];
  uint32_t base[16];
  uint32_t bt_status;
  uint16_t rev_of[320];
  uint8_t lens[320];
  uint8_t cl_lens[20];
};
constexpr uint32_t kTableImage = offsetof(HuffLds, offs);
// dyn_header_par's per-lane symbol scratch (ClLds) may alias lit[]: the
// litlen table is built only after the code lengths are decoded
static_assert(kTableImage % 16 == 0, "table image is copied in 16 B units");
static_assert(kTableImage == kHuffTableImage, "hbam_device.h kHuffTableImage must match HuffLds");

// A code of length l fills 2^(root - l) root entries: codes with l <= root -
// kFillWave are filled by the whole wave together, longer ones by their lane.
#ifndef HBAM_FILL_WAVE
#define HBAM_FILL_WAVE 6
#endif
constexpr int kFillWave = HBAM_FILL_WAVE;

// mode 0 litlen, 1 distance, 2 code-length codes
__device__ __forceinline__ uint32_t make_entry(int mode, uint32_t s, uint32_t len) {
  if (mode == 0) {
    if (s < 256) return (len << 16) | (1u << 24) | s;
    if (s == 256) return (len << 16) | (K_EOB << 26);
    if (s < 286) {
      const uint32_t i = s - 257;
      return (len << 16) | (K_LEN << 26) | ((uint32_t)kLenExtra[i] << 9) | (uint32_t)kLenBase[i];
    }
    return (len << 16) | kBadEntry;
  }
  if (mode == 1) {
    if (s < 30) return (len << 16) | ((uint32_t)kDistExtra[s] << 21) | (uint32_t)kDistBase[s];
    return (len << 16) | kBadEntry;
  }
  return (len << 16) | s;
}

// Canonical Huffman table build by ONE wave (wave 0 of the workgroup; the
// other waves wait at the caller's barrier).  Validity follows
// zlib inflate_table: over-subscribed -> error; incomplete -> error unless
// the only code has length 1 (LENS/DISTS); no codes -> all-invalid table
// (DISTS) or error (CODES).  Returns 0 on success.  Per-length state lives in
// LDS (not in unrolled SGPR arrays) to keep the decode loop's registers free.
// Callers must rfl() the result: a call's return value is divergent to the
// compiler, and one divergent branch at the call site turns the whole decode
// state into VGPRs with exec-masked control flow.
__device__ __attribute__((noinline)) int build_table(HuffLds& L, const uint8_t* lens, int nsym, int root, int mode,
                                                     uint32_t* tab, uint32_t* cnt, uint16_t* sorted, uint32_t* sub,
                                                     int subcap) {
  const uint32_t lane = lane_id();
  // counts per code length by ballots, then the Kraft check, the canonical
  // offsets and first codes as wave-uniform arithmetic (LDS atomics and a
  // one-lane loop over LDS cost ~3 K cycles per table)
  uint32_t cntv[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) cntv[q] = 0;
  for (int c0 = 0; c0 < nsym; c0 += 64) {
    const int s = c0 + (int)lane;
    const uint32_t l = s < nsym ? lens[s] : 0;
#pragma unroll
    for (uint32_t q = 1; q < 16; ++q) cntv[q] += (uint32_t)__popcll(__ballot(l == q));
  }
  int left = 1, maxl = 0;
  bool over = false;
  uint32_t o = 0, code = 0, prev = 0, my_cnt = 0, my_off = 0, my_first = 0;
#pragma unroll
  for (uint32_t l = 1; l < 16; ++l) {
    const uint32_t c = cntv[l];
    left = (left << 1) - (int)c;
    maxl = c ? (int)l : maxl;
    over = over || left < 0;
    code = (code + prev) << 1;
    my_cnt = lane == l ? c : my_cnt;
    my_off = lane == l ? o : my_off;
    my_first = lane == l ? code : my_first;
    o += c;
    prev = c;
  }
  if (lane < 16) {
    cnt[lane] = my_cnt;
    L.offs[lane] = my_off;
    L.firstc[lane] = my_first;
  }
  uint32_t st = 0;
  if (over) st = 1;
  else if (maxl == 0) st = mode == 2 ? 1 : 2;
  else if (left > 0 && (mode == 2 || maxl != 1)) st = 1;
  for (int i = lane; i < (1 << root); i += 64) tab[i] = kBadEntry;
  wave_sync();
  if (st == 1) return 1;
  if (st == 2) return 0;  // no codes: all-invalid table
  const uint32_t rmask = (1u << root) - 1;
  const uint64_t ltmask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  bool any_long = false;
  // next canonical rank per code length: wave-uniform, kept in registers (an
  // LDS counter costs a dependent LDS round trip per length and group)
  uint32_t basev[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) basev[q] = 0;
  for (int c0 = 0; c0 < nsym; c0 += 64) {
    const int s = c0 + (int)lane;
    const uint32_t l = s < nsym ? lens[s] : 0;
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t q = 1; q < 16; ++q) {
      const uint64_t m = __ballot(l == q);
      rank = l == q ? basev[q] + (uint32_t)__popcll(m & ltmask) : rank;
      basev[q] += (uint32_t)__popcll(m);
    }
    uint32_t rev = 0, e = 0;
    if (l) {
      sorted[L.offs[l] + rank] = (uint16_t)s;
      const uint32_t code = L.firstc[l] + rank;
      rev = __brev(code) >> (32 - l);
      L.rev_of[s] = (uint16_t)rev;
      if ((int)l <= root) {
        e = make_entry(mode, (uint32_t)s, l);
        // a code that fills fewer than 64 root entries fills them itself; the
        // wave fills the wider ones together below (a lane alone took up to
        // 2^(root - l) dependent trips, and the wave waited for the longest)
        if ((int)l > root - kFillWave)
          for (uint32_t i = rev; i < (1u << root); i += (1u << l)) tab[i] = e;
      } else {
        atomicMax(&tab[rev & rmask], kLongTag | (l - (uint32_t)root));  // widest sub-table under the prefix
        any_long = true;
      }
    }
    for (uint64_t wm = __ballot(l != 0 && (int)l <= root - kFillWave); wm; wm &= wm - 1) {
      const int src = __ffsll((long long)wm) - 1;
      const uint32_t wl = (uint32_t)__builtin_amdgcn_readlane((int)l, src);  // src is wave-uniform
      const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)rev, src);
      const uint32_t we = (uint32_t)__builtin_amdgcn_readlane((int)e, src);
      for (uint32_t k = lane; k < (1u << (root - (int)wl)); k += 64) tab[wr + (k << wl)] = we;
    }
  }
  wave_sync();
  if (__ballot(any_long) == 0) return 0;
  // sub-table bases: exclusive scan of the sub-table sizes in root-index order
  uint32_t used = 0;
  for (int c0 = 0; c0 < (1 << root); c0 += 64) {
    const uint32_t i = c0 + lane;
    const uint32_t t = tab[i];
    const bool mk = t >= kLongTag;
    const uint32_t bits = t & 15u;
    const uint32_t sz = mk ? (1u << bits) : 0u;
    uint32_t inc = sz;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, 64);
      if (lane >= (uint32_t)d) inc += v;
    }
    const uint32_t base = used + inc - sz;
    if (mk) tab[i] = base + sz <= (uint32_t)subcap ? (kLongEntry | (bits << 16) | base) : (K_SLOW << 26);
    used += (uint32_t)__shfl(inc, 63, 64);
  }
  const uint32_t nused = min(used, (uint32_t)subcap);
  for (uint32_t i = lane; i < nused; i += 64) sub[i] = kBadEntry;
  wave_sync();
  for (int s = lane; s < nsym; s += 64) {
    const uint32_t l = lens[s];
    if ((int)l > root) {
      const uint32_t rev = L.rev_of[s];
      const uint32_t e = tab[rev & rmask];
      if (is_long(e)) {
        const uint32_t b = e & 0xffffu, sb = (e >> 16) & 15u;
        const uint32_t ent = make_entry(mode, (uint32_t)s, l);
        for (uint32_t k = rev >> root; k < (1u << sb); k += 1u << (l - root)) sub[b + k] = ent;
      }
    }
  }
  wave_sync();
  return 0;
}

// The same build with its per-length state and the code lengths in registers
// (k_huff_tables, §7 item 2 of DESIGN.md): ~25 % faster per table, but its
// ~116 VGPRs would spill k_inflate_huff, whose rare inline header path calls
// the LDS-state build_table above.
__device__ __attribute__((noinline)) int build_table_r(HuffLds& L, const uint8_t* lens, int nsym, int root, int mode,
                                                     uint32_t* tab, uint32_t* cnt, uint16_t* sorted, uint32_t* sub,
                                                     int subcap) {
  const uint32_t lane = lane_id();
  // Every symbol's code length stays in registers (nsym <= 320: 5 groups of
  // 64), so do the canonical offsets and first codes (wave-uniform, picked
  // per lane by a select chain): each LDS read on this path is a dependent
  // round trip in a wave that has nothing else to do.
  constexpr int kGroups = 5;
  const int ng = (nsym + 63) >> 6;
  uint32_t lv[kGroups];
#pragma unroll
  for (int g = 0; g < kGroups; ++g) {
    const int s = 64 * g + (int)lane;
    lv[g] = g < ng && s < nsym ? lens[s] : 0u;
  }
  // counts per code length by ballots, then the Kraft check, the canonical
  // offsets and first codes as wave-uniform arithmetic (LDS atomics and a
  // one-lane loop over LDS cost ~3 K cycles per table)
  uint32_t cntv[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) cntv[q] = 0;
#pragma unroll
  for (int g = 0; g < kGroups; ++g) {
    if (g >= ng) break;  // wave-uniform
#pragma unroll
    for (uint32_t q = 1; q < 16; ++q) cntv[q] += (uint32_t)__popcll(__ballot(lv[g] == q));
  }
  int left = 1, maxl = 0;
  bool over = false;
  uint32_t o = 0, code = 0, prev = 0, my_cnt = 0;
  uint32_t offu[16], firstu[16];
  offu[0] = firstu[0] = 0;
#pragma unroll
  for (uint32_t l = 1; l < 16; ++l) {
    const uint32_t c = cntv[l];
    left = (left << 1) - (int)c;
    maxl = c ? (int)l : maxl;
    over = over || left < 0;
    code = (code + prev) << 1;
    my_cnt = lane == l ? c : my_cnt;
    offu[l] = o;
    firstu[l] = code;
    o += c;
    prev = c;
  }
  if (lane < 16) cnt[lane] = my_cnt;
  uint32_t st = 0;
  if (over) st = 1;
  else if (maxl == 0) st = mode == 2 ? 1 : 2;
  else if (left > 0 && (mode == 2 || maxl != 1)) st = 1;
  for (int i = lane; i < (1 << root); i += 64) tab[i] = kBadEntry;
  wave_sync();
  if (st == 1) return 1;
  if (st == 2) return 0;  // no codes: all-invalid table
  const uint32_t rmask = (1u << root) - 1;
  const uint64_t ltmask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  bool any_long = false;
  // next canonical rank per code length: wave-uniform, kept in registers (an
  // LDS counter costs a dependent LDS round trip per length and group)
  uint32_t basev[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) basev[q] = 0;
  uint32_t revv[kGroups];
#pragma unroll
  for (int g = 0; g < kGroups; ++g) {
    revv[g] = 0;
    if (g >= ng) break;  // wave-uniform
    const int s = 64 * g + (int)lane;
    const uint32_t l = lv[g];
    uint32_t rank = 0, off = 0, first = 0;
#pragma unroll
    for (uint32_t q = 1; q < 16; ++q) {
      const uint64_t m = __ballot(l == q);
      rank = l == q ? basev[q] + (uint32_t)__popcll(m & ltmask) : rank;
      off = l == q ? offu[q] : off;
      first = l == q ? firstu[q] : first;
      basev[q] += (uint32_t)__popcll(m);
    }
    uint32_t rev = 0, e = 0;
    if (l) {
      sorted[off + rank] = (uint16_t)s;
      rev = __brev(first + rank) >> (32 - l);
      revv[g] = rev;
      if ((int)l <= root) {
        e = make_entry(mode, (uint32_t)s, l);
        // a code that fills fewer than 64 root entries fills them itself; the
        // wave fills the wider ones together below (a lane alone took up to
        // 2^(root - l) dependent trips, and the wave waited for the longest)
        if ((int)l > root - kFillWave)
          for (uint32_t i = rev; i < (1u << root); i += (1u << l)) tab[i] = e;
      } else {
        atomicMax(&tab[rev & rmask], kLongTag | (l - (uint32_t)root));  // widest sub-table under the prefix
        any_long = true;
      }
    }
    for (uint64_t wm = __ballot(l != 0 && (int)l <= root - kFillWave); wm; wm &= wm - 1) {
      const int src = __ffsll((long long)wm) - 1;
      const uint32_t wl = (uint32_t)__builtin_amdgcn_readlane((int)l, src);  // src is wave-uniform
      const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)rev, src);
      const uint32_t we = (uint32_t)__builtin_amdgcn_readlane((int)e, src);
      for (uint32_t k = lane; k < (1u << (root - (int)wl)); k += 64) tab[wr + (k << wl)] = we;
    }
  }
  wave_sync();
  if (__ballot(any_long) == 0) {
    return 0;
  }
  // sub-table bases: exclusive sum of the sub-table sizes in root-index
  // order.  A table has a handful of long-code prefixes, so the marked
  // entries of each 64-entry chunk are walked in lane order (a 6-step
  // shuffle scan of every chunk, ds_bpermute each step, took ~12 K cycles);
  // the root entries are read all at once first
  constexpr int kChunks = (1 << kLitRoot) / 64;
  const int nch = (1 << root) >> 6;
  uint32_t tv[kChunks];
#pragma unroll
  for (int c = 0; c < kChunks; ++c) tv[c] = c < nch ? tab[64 * c + lane] : 0u;
  uint32_t used = 0;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const uint32_t t = tv[c];  // 0 past the root table: no marks
    for (uint64_t mm = __ballot(t >= kLongTag); mm; mm &= mm - 1) {
      const int j = __ffsll((long long)mm) - 1;
      const uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)t, j) & 15u;
      const uint32_t sz = 1u << bits;
      if ((int)lane == j)
        tab[64 * c + lane] = used + sz <= (uint32_t)subcap ? (kLongEntry | (bits << 16) | used) : (K_SLOW << 26);
      used += sz;
    }
  }
  const uint32_t nused = min(used, (uint32_t)subcap);
  for (uint32_t i = lane; i < nused; i += 64) sub[i] = kBadEntry;
  wave_sync();
#pragma unroll
  for (int g = 0; g < kGroups; ++g) {
    if (g >= ng) break;  // wave-uniform
    const uint32_t l = lv[g];
    if ((int)l > root) {
      const int s = 64 * g + (int)lane;
      const uint32_t rev = revv[g];
      const uint32_t e = tab[rev & rmask];
      if (is_long(e)) {
        const uint32_t b = e & 0xffffu, sb = (e >> 16) & 15u;
        const uint32_t ent = make_entry(mode, (uint32_t)s, l);
        for (uint32_t k = rev >> root; k < (1u << sb); k += 1u << (l - root)) sub[b + k] = ent;
      }
    }
  }
  wave_sync();
  return 0;
}

// Fold two consecutive literals into one litlen entry when both codes fit in
// the 10-bit index (the common case for quality/sequence bytes).
__device__ __attribute__((noinline)) void pair_literals(HuffLds& L) {
  const uint32_t lane = lane_id();
  uint32_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t i = lane + 64u * j;
    const uint32_t e1 = L.lit[i];
    v[j] = e1;
    const uint32_t l1 = (e1 >> 16) & 31;
    if (e1 < kKindLit && l1 < (uint32_t)kLitRoot) {
      const uint32_t e2 = L.lit[i >> l1];
      const uint32_t l2 = (e2 >> 16) & 31;
      if (e2 < kKindLit && l2 + l1 <= (uint32_t)kLitRoot)
        v[j] = ((l1 + l2) << 16) | (2u << 24) | (e1 & 0xffu) | ((e2 & 0xffu) << 8);
    }
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < 16; ++j) L.lit[lane + 64u * j] = v[j];
  wave_sync();
}

// puff-style canonical decode (sub-table overflow, split literal pairs: rare).
template <bool UNIFORM>
__device__ uint32_t canon_decode(uint64_t bits, const uint32_t* cnt, const uint16_t* sorted, int mode) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len < 16; ++len) {
    code |= (int)(bits & 1);
    bits >>= 1;
    const int count = UNIFORM ? (int)rfl(cnt[len]) : (int)cnt[len];
    if (code - count < first) {
      const uint32_t s = UNIFORM ? rfl(sorted[index + (code - first)]) : sorted[index + (code - first)];
      return make_entry(mode, s, (uint32_t)len);
    }
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return kBadEntry;
}

template <bool UNIFORM>
__device__ __forceinline__ uint32_t lit_lookup(const HuffLds& L, uint64_t b) {
  uint32_t e = L.lit[(uint32_t)b & ((1u << kLitRoot) - 1)];
  if (UNIFORM) e = rfl(e);
  if (is_long(e)) {
    e = L.litsub[(e & 0xffffu) + ((uint32_t)(b >> kLitRoot) & ((1u << ((e >> 16) & 15u)) - 1))];
    if (UNIFORM) e = rfl(e);
  } else if ((e >> 26) == K_SLOW) {
    e = canon_decode<UNIFORM>(b, L.cnt_lit, L.sort_lit, 0);
  }
  return e;
}
template <bool UNIFORM>
__device__ __forceinline__ uint32_t dist_lookup(const HuffLds& L, uint64_t b) {
  uint32_t d = L.dist[(uint32_t)b & ((1u << kDistRoot) - 1)];
  if (UNIFORM) d = rfl(d);
  if (is_long(d)) {
    d = L.distsub[(d & 0xffffu) + ((uint32_t)(b >> kDistRoot) & ((1u << ((d >> 16) & 15u)) - 1))];
    if (UNIFORM) d = rfl(d);
  } else if ((d >> 26) == K_SLOW) {
    d = canon_decode<UNIFORM>(b, L.cnt_dist, L.sort_dist, 1);
  }
  return d;
}

// lane_decode exit events (EV_MERGE: the sync walk reached a boundary of the
// lane's speculative walk)
enum : uint32_t { EV_STOP = 0, EV_EOB = 1, EV_INPUT = 2, EV_ERR = 3, EV_FULLX = 4, EV_FULLO = 5, EV_MERGE = 6 };
enum { LD_SPEC = 0, LD_SYNC = 1, LD_EMIT = 2 };

// Boundaries of a lane's speculative walk: p[k] = bit position after symbol
// kMergeFirst << k, b[k] = output bytes decoded up to there (~0u = not reached).
#ifndef HBAM_MERGE_FIRST
#define HBAM_MERGE_FIRST 4
#endif
constexpr uint32_t kMergeFirst = HBAM_MERGE_FIRST;  // power of two
static_assert((kMergeFirst & (kMergeFirst - 1)) == 0, "kMergeFirst: a power of two");
// Slices shorter than this many bits (a short last DEFLATE block) take their
// boundaries at kMergeFirst / 2 << k instead (0: never)
#ifndef HBAM_MERGE_SHORT_BITS
#define HBAM_MERGE_SHORT_BITS 400
#endif
constexpr uint32_t kMergeShortBits = HBAM_MERGE_SHORT_BITS;
#ifndef HBAM_MERGE_TINY_BITS
#define HBAM_MERGE_TINY_BITS 0
#endif
constexpr uint32_t kMergeTinyBits = HBAM_MERGE_TINY_BITS;  // ... kMergeFirst / 4 << k below this
struct MergePts {
  uint32_t p0, p1, p2, p3;
  uint32_t b0, b1, b2, b3;
};

// 16 B token store with 4 B alignment (global memory; unaligned mode).
struct __attribute__((packed, aligned(4))) Tok4 {
  uint32_t a, b, c, d;
};

// Decode from bit `a` while the position is below `stop` (bit positions are
// relative to the 16 B-aligned LDS image W; E = end of CDATA).  Returns the
// event that ended the walk; x = position reached, nt/nb = tokens/bytes
// decoded.
//   LD_SPEC records the first boundaries in mp;
//   LD_SYNC stops with EV_MERGE (mj = index) when it reaches one of them;
//   LD_EMIT writes tokens to tok[0..nt) and applies the output-space rules with
//           the output position of the first token = out0.
template <int MODE>
__device__ __forceinline__ uint32_t lane_decode(const HuffLds& L, const uint32_t* __restrict__ W, uint32_t a,
                                                uint32_t stop, uint32_t E, uint32_t& x, uint32_t& nt, uint32_t& nb,
                                                MergePts& mp, uint32_t& mj, uint32_t* __restrict__ tok,
                                                uint32_t out0, uint32_t isize, uint32_t mf = kMergeFirst) {
  constexpr bool EMIT = MODE == LD_EMIT;
  uint32_t wd, cnt, nx;
  uint64_t buf;
#define LSEEK(p)                                                    \
  do {                                                              \
    wd = (p) >> 5;                                                  \
    buf = (((uint64_t)W[wd + 1] << 32) | W[wd]) >> ((p) & 31);      \
    cnt = 64 - ((p) & 31);                                          \
    wd += 2;                                                        \
    nx = W[wd];                                                     \
  } while (0)
  LSEEK(a);
  uint32_t pos = a, ev = EV_STOP;
  uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, fill = 0;  // EMIT: pending tokens
  nt = 0;
  nb = 0;
  if (MODE == LD_SPEC) {
    mp.p0 = mp.p1 = mp.p2 = mp.p3 = ~0u;
    mp.b0 = mp.b1 = mp.b2 = mp.b3 = ~0u;
  }
#define LREFILL()                        \
  do {                                   \
    if (cnt <= 32) {                     \
      buf |= (uint64_t)nx << cnt;        \
      cnt += 32;                         \
      ++wd;                              \
      nx = W[wd];                        \
    }                                    \
  } while (0)
#define LCONSUME(n)  \
  do {               \
    buf >>= (n);     \
    cnt -= (n);      \
    pos += (n);      \
  } while (0)
#define LCOMMIT(t_, len_)                                                                   \
  do {                                                                                      \
    if (EMIT) {                                                                             \
      q0 = fill == 0 ? (t_) : q0;                                                           \
      q1 = fill == 1 ? (t_) : q1;                                                           \
      q2 = fill == 2 ? (t_) : q2;                                                           \
      q3 = (t_);                                                                            \
      if (++fill == 4) {                                                                    \
        *reinterpret_cast<Tok4*>(tok + nt - 3) = Tok4{q0, q1, q2, q3};                      \
        fill = 0;                                                                           \
      }                                                                                     \
    }                                                                                       \
    ++nt;                                                                                   \
    nb += (len_);                                                                           \
    if (MODE == LD_SPEC && (nt & (nt - 1)) == 0 && nt >= mf && nt <= 8 * mf) {                   \
      /* boundaries after symbols F, 2F, 4F, 8F: the speculative walk has */                \
      /* usually joined the true path by the later ones */                                  \
      mp.p0 = nt == mf ? pos : mp.p0;                                              \
      mp.b0 = nt == mf ? nb : mp.b0;                                               \
      mp.p1 = nt == 2 * mf ? pos : mp.p1;                                          \
      mp.b1 = nt == 2 * mf ? nb : mp.b1;                                           \
      mp.p2 = nt == 4 * mf ? pos : mp.p2;                                          \
      mp.b2 = nt == 4 * mf ? nb : mp.b2;                                           \
      mp.p3 = nt == 8 * mf ? pos : mp.p3;                                          \
      mp.b3 = nt == 8 * mf ? nb : mp.b3;                                           \
    }                                                                                       \
  } while (0)
  // Fast path: while a whole symbol (<= 15+5+15+13 = 48 bits) fits before E,
  // no CDATA-end checks are needed; literal and length/distance symbols are
  // decoded with selects instead of divergent branches (the wave mixes both in
  // nearly every step).  End-of-block, invalid codes and (EMIT) distances
  // beyond the output leave it; the slow path below re-decodes that symbol
  // from `pos` with every zlib check.
  const uint32_t fast_end = E >= 48 ? min(stop, E - 47) : 0u;
  for (;;) {
    bool merged = false;
    // Every lane peeks the 64 bits at `pos` from three words (no bit-buffer
    // refills).  The loop runs with the wave's exec mask unchanged until no
    // lane is active (one scalar branch per symbol): a lane that has left
    // (act = 0) or meets a symbol the fast path does not take (ok = 0) only
    // computes, every update is a select.  The branchy form paid an exec-mask
    // update per branch on the scalar unit that the CU's 16 waves share
    // (SQ_INSTS_SALU ~ 0.8 x SQ_INSTS_VALU, the issue limit of the kernel).
    // go(p): inside the fast region; SYNC: hit = p is a boundary of the lane's
    // speculative walk (the walks share every symbol from there on; the min
    // of the xors is 0 iff one matches).  & rather than &&: no branches.
    auto fast_go = [&](uint32_t p, uint32_t bytes, bool& hit) -> bool {
      hit = false;
      if (MODE == LD_SYNC) hit = min(min(p ^ mp.p0, p ^ mp.p1), min(p ^ mp.p2, p ^ mp.p3)) == 0;
      return (p < fast_end) & (!EMIT | (out0 + bytes < isize));
    };
    bool hit0;
    const bool g0 = fast_go(pos, nb, hit0);
    merged = g0 & hit0;
    bool act = g0 & !hit0;
    uint32_t it = 0, ucp = mf;  // iterations of this loop, next checkpoint iteration (wave-uniform)
    if (__builtin_amdgcn_ballot_w64(act)) do {
      const uint32_t wd = pos >> 5, sh = pos & 31;
      const uint32_t w0 = W[wd], w1 = W[wd + 1], w2 = W[wd + 2];
      const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh);
      const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, sh);
      uint32_t e = L.lit[lo & ((1u << kLitRoot) - 1)];
      {  // a code longer than the root (rare): every lane reads, long ones keep it
        const bool lg = is_long(e);
        if (__builtin_amdgcn_ballot_w64(lg)) {
          const uint32_t es = L.litsub[min((e & 0xffffu) + __builtin_amdgcn_ubfe(lo, kLitRoot, (e >> 16) & 15u),
                                           (uint32_t)kLitSubCap - 1)];  // in bounds for the lanes that drop it
          e = lg ? es : e;
        }
      }
      // kind 0 literal, 1 length: isl = bit 26; kind > 1 leaves the fast path
      const uint32_t isl = (e >> 26) & 1u;
      const uint32_t n1 = (e >> 16) & 31;
      const uint32_t ex = __builtin_amdgcn_ubfe(e, 9, 4 * isl);
      // literal: e >> 24 bytes; length: base + ex extra bits (ubfe of 0 bits is 0)
      const uint32_t len = (isl ? (e & 511) : (e >> 24)) + __builtin_amdgcn_ubfe(lo, n1, ex);
      const uint32_t c1 = n1 + ex;  // <= 20: the distance code starts inside lo
      const uint32_t b2 = __builtin_amdgcn_alignbit(hi, lo, c1);
      uint32_t d = L.dist[b2 & ((1u << kDistRoot) - 1)];
      {
        const bool lg = is_long(d);
        if (__builtin_amdgcn_ballot_w64(lg)) {
          const uint32_t ds = L.distsub[min((d & 0xffffu) + __builtin_amdgcn_ubfe(b2, kDistRoot, (d >> 16) & 15u),
                                            (uint32_t)kDistSubCap - 1)];
          d = lg ? ds : d;
        }
      }
      const uint32_t dn = (d >> 16) & 31, dx = (d >> 21) & 15;
      const uint32_t dist = (d & 0x7fff) + __builtin_amdgcn_ubfe(b2, dn, dx);
      // not taken here (the slow path decodes that symbol): an EOB / invalid /
      // canonical-decode entry (e >= 2 << 26), an invalid or canonical-decode
      // distance entry for a length (d >= 1 << 26: kinds K_BAD and K_SLOW),
      // (EMIT) a distance before the block start
      bool bad = (e >= (2u << 26)) | ((isl != 0) & (d >= kKindLit));
      if (EMIT) bad |= (isl != 0) & (out0 + nb < dist);
      const bool upd = act & !bad;
      const uint32_t tm = 0x80000000u | ((dist - 1) << 16) | len, tl = e & 0x0300ffffu;
      const uint32_t t = tl ^ ((tm ^ tl) & (0u - isl));
      const uint32_t npos = pos + c1 + ((dn + dx) & (0u - isl));
      pos = upd ? npos : pos;
      nb += upd ? len : 0u;
      if (EMIT) {
        const uint32_t fs = upd ? fill : 7u;  // the queue slot this token takes (7: none)
        q0 = fs == 0 ? t : q0;
        q1 = fs == 1 ? t : q1;
        q2 = fs == 2 ? t : q2;
        q3 = upd ? t : q3;
        if (fs == 3) *reinterpret_cast<Tok4*>(tok + nt - 3) = Tok4{q0, q1, q2, q3};
        fill = upd ? (fill + 1) & 3u : fill;
      }
      nt += upd ? 1u : 0u;
      ++it;
      if (MODE == LD_SPEC && it == ucp) {
        // boundaries after symbols F, 2F, 4F, 8F, tested at the iteration of
        // that number (uniform): a lane that entered this loop with nt = 0 and
        // decoded a symbol in every iteration has nt == it.  A lane that
        // re-entered after the slow path records only where the counts
        // agree; a missing boundary costs its sync walk time, not a result.
        const bool cp = upd & (nt == it);
        if (it == mf) { mp.p0 = cp ? pos : mp.p0; mp.b0 = cp ? nb : mp.b0; }
        if (it == 2 * mf) { mp.p1 = cp ? pos : mp.p1; mp.b1 = cp ? nb : mp.b1; }
        if (it == 4 * mf) { mp.p2 = cp ? pos : mp.p2; mp.b2 = cp ? nb : mp.b2; }
        if (it == 8 * mf) { mp.p3 = cp ? pos : mp.p3; mp.b3 = cp ? nb : mp.b3; }
        ucp = it == 8 * mf ? 0u : 2 * it;
      }
      bool hit;
      const bool g = fast_go(pos, nb, hit);
      merged = merged | (upd & g & hit);
      act = upd & g & !hit;
    } while (__builtin_amdgcn_ballot_w64(act));
    if (MODE == LD_SYNC && merged) {
      const bool h0 = pos == mp.p0, h1 = pos == mp.p1, h2 = pos == mp.p2;
      mj = h0 ? 0u : h1 ? 1u : h2 ? 2u : 3u;
    }
    if (MODE == LD_SYNC && merged) {
      ev = EV_MERGE;
      break;
    }
    // ---- slow path: one symbol with every check (or the end of the slice)
    if (pos >= stop) break;
    LSEEK(pos);
    if (MODE == LD_SYNC) {
      const bool h0 = pos == mp.p0, h1 = pos == mp.p1, h2 = pos == mp.p2, h3 = pos == mp.p3;
      if (h0 | h1 | h2 | h3) {
        mj = h0 ? 0u : h1 ? 1u : h2 ? 2u : 3u;
        ev = EV_MERGE;
        break;
      }
    }
    if (EMIT && out0 + nb >= isize) {
      ev = (out0 + nb == isize) ? EV_FULLX : EV_FULLO;
      break;
    }
    LREFILL();
    uint32_t e = lit_lookup<false>(L, buf);
    uint32_t n1 = (e >> 16) & 31;
    uint32_t t, len;
    if (e < kKindLit) {
      if (pos + n1 > E) {  // a pair may straddle the end: decode the first literal alone
        if ((e >> 24) == 2u) {
          e = canon_decode<false>(buf, L.cnt_lit, L.sort_lit, 0);
          n1 = (e >> 16) & 31;
        }
        if (pos + n1 > E) { ev = EV_INPUT; break; }
      }
      t = e & 0x0300ffffu;
      len = e >> 24;
      LCONSUME(n1);
    } else {
      const uint32_t k = e >> 26;
      if (k == K_LEN) {
        const uint32_t ex = (e >> 9) & 15;
        if (pos + n1 + ex > E) { ev = EV_INPUT; break; }
        len = (e & 511) + ((uint32_t)(buf >> n1) & ((1u << ex) - 1));
        LCONSUME(n1 + ex);
        LREFILL();
        const uint32_t d = dist_lookup<false>(L, buf);
        const uint32_t dn = (d >> 16) & 31;
        if (d >= kKindLit) {  // invalid distance code
          ev = (pos + max(dn, 1u) > E) ? EV_INPUT : EV_ERR;
          break;
        }
        const uint32_t dx = (d >> 21) & 15;
        if (pos + dn + dx > E) { ev = EV_INPUT; break; }
        const uint32_t dist = (d & 0x7fff) + ((uint32_t)(buf >> dn) & ((1u << dx) - 1));
        LCONSUME(dn + dx);
        if (EMIT && dist > out0 + nb) { ev = EV_ERR; break; }  // invalid distance too far back
        t = 0x80000000u | ((dist - 1) << 16) | len;
      } else if (k == K_EOB) {
        if (pos + n1 > E) { ev = EV_INPUT; break; }
        LCONSUME(n1);
        ev = EV_EOB;
        break;
      } else {  // invalid literal/length code
        ev = (pos + max(n1, 1u) > E) ? EV_INPUT : EV_ERR;
        break;
      }
    }
    LCOMMIT(t, len);
  }
#undef LSEEK
#undef LREFILL
#undef LCONSUME
#undef LCOMMIT
  if (EMIT && fill) {  // the 1..3 tokens not yet stored
    uint32_t* p = tok + nt - fill;
    p[0] = q0;
    if (fill > 1) p[1] = q1;
    if (fill > 2) p[2] = q2;
  }
  x = pos;
  return ev;
}

// Inclusive wave scan on DPP (VALU lane moves, no LDS round trip): Hillis-Steele
// inside each 16-lane row, then row_bcast:15 / row_bcast:31 carry the row totals.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Inclusive wave max-scan on DPP (as wave_incl_scan_dpp; 0 is the identity).
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));   // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));   // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));   // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));   // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// Workgroup-wide helpers for the phase-A workgroup (all threads call them in
// uniform control flow; each ends with a barrier so `red` can be reused).
__device__ __forceinline__ uint32_t wg_any(bool p, uint32_t* red) {
  const uint32_t w = threadIdx.x >> 6;
  const uint64_t b = __ballot(p);
  if (lane_id() == 0) red[w] = b != 0;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < kHuffWaves; ++i) r |= red[i];
  __syncthreads();
  return r;
}
__device__ __forceinline__ uint32_t wg_min(uint32_t v, uint32_t* red) {
  const uint32_t w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d, 64));
  if (lane_id() == 0) red[w] = v;
  __syncthreads();
  uint32_t r = 0xffffffffu;
#pragma unroll
  for (int i = 0; i < kHuffWaves; ++i) r = min(r, red[i]);
  __syncthreads();
  return r;
}
// exclusive scans of (u, v) over the workgroup
__device__ __forceinline__ void wg_excl_scan2(uint32_t u, uint32_t v, uint32_t* red, uint32_t& eu, uint32_t& ev) {
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t iu = wave_incl_scan(u), iv = wave_incl_scan(v);
  if (lane_id() == 63) {
    red[w] = iu;
    red[kHuffWaves + w] = iv;
  }
  __syncthreads();
  uint32_t ou = 0, ov = 0;
#pragma unroll
  for (int i = 0; i < kHuffWaves; ++i) {
    ou += (uint32_t)i < w ? red[i] : 0u;
    ov += (uint32_t)i < w ? red[kHuffWaves + i] : 0u;
  }
  __syncthreads();
  eu = ou + iu - u;
  ev = ov + iv - v;
}

// Wave-uniform bit reader over a 16 B-aligned LDS image (block headers, code
// lengths, lookahead).  Values are readfirstlane'd so the state stays in SGPRs.
struct SReader {
  const uint32_t* W;
  uint64_t buf;
  uint32_t cnt, wd;
  __device__ __forceinline__ void seek(uint32_t p) {
    wd = p >> 5;
    buf = (((uint64_t)rfl(W[wd + 1]) << 32) | rfl(W[wd])) >> (p & 31);
    cnt = 64 - (p & 31);
    wd += 2;
  }
  __device__ __forceinline__ void fill() {
    if (cnt <= 32) {
      buf |= (uint64_t)rfl(W[wd]) << cnt;
      cnt += 32;
      ++wd;
    }
  }
  __device__ __forceinline__ uint32_t pos() const { return 32u * wd - cnt; }
  __device__ __forceinline__ void consume(uint32_t n) {
    buf >>= n;
    cnt -= n;
  }
};

// Dynamic-Huffman block header after BTYPE: code-length code, code lengths,
// litlen / distance tables (+ literal pairing).  Run by one wave.  Returns
// DH_OK, DH_TRUNC (a field does not fit before bit E) or kErrIO
// (DataFormatException: bad counts, over/under-subscribed codes, a repeat with
// no previous length, no end-of-block code).
enum : int { DH_OK = 0, DH_TRUNC = -1 };
__device__ __forceinline__ int dyn_header(HuffLds& L, SReader& R, uint32_t E) {
  const uint32_t lane = lane_id();
  R.fill();
  if (R.pos() + 14 > E) return DH_TRUNC;
  const uint32_t hlit = ((uint32_t)R.buf & 31) + 257;
  const uint32_t hdist = ((uint32_t)(R.buf >> 5) & 31) + 1;
  const uint32_t hclen = ((uint32_t)(R.buf >> 10) & 15) + 4;
  R.consume(14);
  if (hlit > 286 || hdist > 30) return kErrIO;
  if (R.pos() + 3 * hclen > E) return DH_TRUNC;
  if (lane < 20) L.cl_lens[lane] = 0;
  wave_sync();
  for (uint32_t i = 0; i < hclen; ++i) {
    R.fill();
    const uint32_t v = (uint32_t)R.buf & 7;
    R.consume(3);
    if (lane == 0) L.cl_lens[kClOrder[i]] = (uint8_t)v;
  }
  wave_sync();
  if (rfl(build_table(L, L.cl_lens, 19, 7, 2, L.dist, L.cnt_dist, L.sort_dist, nullptr, 0))) return kErrIO;
  const uint32_t ntot = hlit + hdist;
  uint32_t i = 0, last = 0;
  while (i < ntot) {
    R.fill();
    const uint32_t e = rfl(L.dist[(uint32_t)R.buf & 127]);
    const uint32_t nbits = (e >> 16) & 31;
    if (R.pos() + nbits > E) return DH_TRUNC;
    const uint32_t sym = e & 0xffff;
    uint32_t rep, val, xb = 0;
    if (sym < 16) {
      rep = 1;
      val = sym;
    } else if (sym == 16) {
      xb = 2;
      rep = 3 + ((uint32_t)(R.buf >> nbits) & 3);
      val = last;
    } else if (sym == 17) {
      xb = 3;
      rep = 3 + ((uint32_t)(R.buf >> nbits) & 7);
      val = 0;
    } else {
      xb = 7;
      rep = 11 + ((uint32_t)(R.buf >> nbits) & 127);
      val = 0;
    }
    if (R.pos() + nbits + xb > E) return DH_TRUNC;
    if (sym == 16 && i == 0) return kErrIO;  // repeat with no previous length
    R.consume(nbits + xb);
    if (i + rep > ntot) return kErrIO;
    for (uint32_t j = lane; j < rep; j += 64) L.lens[i + j] = (uint8_t)val;
    i += rep;
    last = val;
  }
  wave_sync();
  if (rfl(L.lens[256]) == 0) return kErrIO;
  if (rfl(build_table(L, L.lens, (int)hlit, kLitRoot, 0, L.lit, L.cnt_lit, L.sort_lit, L.litsub, kLitSubCap)) ||
      rfl(build_table(L, L.lens + hlit, (int)hdist, kDistRoot, 1, L.dist, L.cnt_dist, L.sort_dist, L.distsub,
                      kDistSubCap)))
    return kErrIO;
  pair_literals(L);
  return DH_OK;
}

// Expected compressed bits of a non-final DEFLATE block, from its code
// lengths (symbol probabilities taken as 2^-length): zlib ends a block after
// lit_bufsize - 1 = 16383 symbols (deflate.c _tr_tally at the default
// memLevel 8), literals and length/distance pairs alike.  It sizes the first
// all-lane pass over the block, so that the slices do not reach far into the
// next block (decoded there with the wrong tables and thrown away); only the
// speed depends on it -- a short guess continues with another pass.  All 64
// lanes of a wave call it; lens[0..hlit) litlen, lens[hlit..hlit+hdist) dist.
constexpr uint32_t kZlibBlockSymbols = 16383;
__device__ uint32_t block_bits_estimate(const uint8_t* lens, uint32_t hlit, uint32_t hdist) {
  const uint32_t lane = lane_id();
  float wl = 0.f, al = 0.f, wlen = 0.f, wd = 0.f, ad = 0.f;
  for (uint32_t s = lane; s < hlit; s += 64) {
    const uint32_t l = lens[s];
    if (l == 0 || s == 256) continue;
    const float w = ldexpf(1.0f, -(int)l);
    wl += w;
    if (s < 256) {
      al += w * (float)l;
    } else if (s < 286) {
      al += w * (float)(l + kLenExtra[s - 257]);
      wlen += w;
    }
  }
  for (uint32_t d = lane; d < hdist && d < 30; d += 64) {
    const uint32_t l = lens[hlit + d];
    if (l == 0) continue;
    const float w = ldexpf(1.0f, -(int)l);
    wd += w;
    ad += w * (float)(l + kDistExtra[d]);
  }
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) {
    wl += __shfl_xor(wl, k, 64);
    al += __shfl_xor(al, k, 64);
    wlen += __shfl_xor(wlen, k, 64);
    wd += __shfl_xor(wd, k, 64);
    ad += __shfl_xor(ad, k, 64);
  }
  const float edist = wd > 0.f ? ad / wd : 0.f;
  const float per_sym = wl > 0.f ? (al + wlen * edist) / wl : 8.f;
  return rfl((uint32_t)fminf((float)kZlibBlockSymbols * per_sym, 1e9f));
}
// End of the first all-lane pass over a DEFLATE block whose symbols start at
// bit b0: an eighth over the estimate (a final block runs to the end).
__device__ __forceinline__ uint32_t pass_end(uint32_t b0, uint32_t est, bool final_blk, uint32_t E) {
  if (final_blk || est == 0) return E;
  const uint64_t e = (uint64_t)b0 + est + (est >> 3) + 1024;
  return e < E ? (uint32_t)e : E;
}

// Dynamic header with the code-length symbols decoded by all 64 lanes of the
// wave (k_huff_tables): lane l speculatively decodes the kClSlice bits from
// p + l*kClSlice of a window, a sync loop restarts slices from their
// predecessor's exit until every lane starts on a true boundary (code-length
// codes are <= 7 bits and resynchronise within a few symbols), then a wave
// scan of the run lengths places every lane's runs in lens[].  Valid headers
// only: any anomaly (bad counts, a repeat with no previous length, a run past
// HLIT+HDIST, bits beyond the staged window) returns DH_TRUNC and the decode
// kernel parses the block inline with dyn_header (the zlib semantics).
constexpr uint32_t kClSlice = 16;
constexpr uint32_t kClMaxSym = kClSlice;  // a slice holds at most one symbol per bit
struct ClLds {
  uint16_t ent[64][kClMaxSym];  // sym | extra << 5 | bits << 12
  uint8_t ex[64][kClSlice];     // k_huff_tables: the slice's exit from each entry offset
};
static_assert(sizeof(ClLds) <= sizeof(HuffLds::lit), "ClLds aliases HuffLds::lit in k_inflate_huff");
static_assert(sizeof(HuffLds::litsub) >= 1024 + 16, "k_huff_tables stages its header bits in litsub");

// Maps of 16 4-bit values (lo: inputs 0-7, hi: 8-15): g <- g o f, i.e.
// g'(e) = g(f(e)).
__device__ __forceinline__ void nib_compose(uint32_t& glo, uint32_t& ghi, uint32_t flo, uint32_t fhi) {
  const uint64_t g = ((uint64_t)ghi << 32) | glo;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    lo |= (uint32_t)(g >> (4u * ((flo >> (4 * e)) & 15u)) & 15u) << (4 * e);
    hi |= (uint32_t)(g >> (4u * ((fhi >> (4 * e)) & 15u)) & 15u) << (4 * e);
  }
  glo = lo;
  ghi = hi;
}

__device__ __forceinline__ uint32_t peek32(const uint32_t* W, uint32_t p) {
  return __builtin_amdgcn_alignbit(W[(p >> 5) + 1], W[p >> 5], p & 31);
}

// build_table_r for k_huff_tables (REG), build_table for k_inflate_huff's inline path
template <bool REG, typename... A>
__device__ __forceinline__ int build_tab(A&&... a) {
  if constexpr (REG) return build_table_r(static_cast<A&&>(a)...);
  else return build_table(static_cast<A&&>(a)...);
}

template <bool REG>
__device__ int dyn_header_par(HuffLds& L, ClLds& C, const uint32_t* __restrict__ W, uint32_t p, uint32_t E,
                              uint32_t* end_pos) {
  const uint32_t lane = lane_id();
  if (p + 14 > E) return DH_TRUNC;
  const uint32_t h = rfl(peek32(W, p));
  const uint32_t hlit = (h & 31) + 257, hdist = ((h >> 5) & 31) + 1, hclen = ((h >> 10) & 15) + 4;
  if (hlit > 286 || hdist > 30) return DH_TRUNC;
  p += 14;
  if (p + 3 * hclen > E) return DH_TRUNC;
  if (lane < 20) L.cl_lens[lane] = 0;
  wave_sync();
  if (lane < hclen) L.cl_lens[kClOrder[lane]] = (uint8_t)(peek32(W, p + 3 * lane) & 7);
  wave_sync();
  p += 3 * hclen;
  if (rfl(build_tab<REG>(L, L.cl_lens, 19, 7, 2, L.dist, L.cnt_dist, L.sort_dist, nullptr, 0))) return DH_TRUNC;
  const uint32_t ntot = hlit + hdist;
  uint32_t done = 0, prevv = 0, have_prev = 0;
  for (;;) {  // windows of 64 * kClSlice bits
    const uint32_t a0 = p + lane * kClSlice, stop = a0 + kClSlice;
    uint32_t a = a0, x = a0, ns = 0;
    if constexpr (REG) {
      // k_huff_tables: the symbol at EVERY bit offset of the slice (16
      // independent lookups), the slice's exit from every entry offset (a
      // backward pass), then the entries of the 64 slices chained on the
      // scalar unit.  The speculative decode + sync loop it replaces
      // restarted 62 of 64 lanes per window, ~21 K cycles per header.
      const bool live0 = a0 + 14 <= E;  // the decode stops at a field that may cross E (monotone in the offset)
      uint64_t win = 0;
      if (live0) win = (((uint64_t)W[(a0 >> 5) + 1] << 32) | W[a0 >> 5]) >> (a0 & 31);
      uint32_t lenv[kClSlice];
#pragma unroll
      for (uint32_t j = 0; j < kClSlice; ++j) {
        const uint32_t b = (uint32_t)(win >> j);
        const uint32_t e = L.dist[b & 127];
        const uint32_t nb = (e >> 16) & 31, sym = e & 0xffff;
        const uint32_t xb = sym < 16 ? 0u : sym == 16 ? 2u : sym == 17 ? 3u : 7u;
        const uint32_t ext = (b >> nb) & ((1u << xb) - 1);
        lenv[j] = nb + xb;
        C.ent[lane][j] = (uint16_t)(sym | (ext << 5) | ((nb + xb) << 12));
      }
      // exit offset (from the slice start) when the decode enters at j; the
      // next slice's entry is exit - kClSlice (<= 14), 15 = stopped at E
      uint32_t glo = 0, ghi = 0;
#pragma unroll
      for (int j = (int)kClSlice - 1; j >= 0; --j) {
        const uint32_t nx = (uint32_t)j + lenv[j];
        uint32_t exj = nx >= kClSlice ? nx : (uint32_t)C.ex[lane][min(nx, kClSlice - 1)];
        if (a0 + (uint32_t)j + 14 > E) exj = (uint32_t)j;
        C.ex[lane][j] = (uint8_t)exj;
        const uint32_t g = exj >= kClSlice ? exj - kClSlice : 15u;
        if (j < 8) glo |= g << (4 * j);
        else ghi |= g << (4 * (j - 8));
      }
      // entry of slice l = F_{l-1}(0), F_l = g_l o ... o g_0: an inclusive
      // DPP scan under composition (15 = stopped stays stopped; a lane with
      // no DPP source takes the identity).  A 64-step scalar chain of
      // readlanes took ~12.8 K cycles per header.
      ghi = (ghi & 0x0fffffffu) | 0xf0000000u;
      constexpr uint32_t kIdLo = 0x76543210u, kIdHi = 0xfedcba98u;
#define CL_SCAN_STEP(ctrl, rmask)                                                                        \
  do {                                                                                                     \
    const uint32_t plo_ = (uint32_t)__builtin_amdgcn_update_dpp((int)kIdLo, (int)glo, ctrl, rmask, 0xf, false); \
    const uint32_t phi_ = (uint32_t)__builtin_amdgcn_update_dpp((int)kIdHi, (int)ghi, ctrl, rmask, 0xf, false); \
    nib_compose(glo, ghi, plo_, phi_); /* g <- g o p: the earlier slices first */                         \
  } while (0)
      CL_SCAN_STEP(0x111, 0xf);  // row_shr:1
      CL_SCAN_STEP(0x112, 0xf);  // row_shr:2
      CL_SCAN_STEP(0x114, 0xf);  // row_shr:4
      CL_SCAN_STEP(0x118, 0xf);  // row_shr:8
      CL_SCAN_STEP(0x142, 0xa);  // row_bcast:15 -> rows 1, 3
      CL_SCAN_STEP(0x143, 0xc);  // row_bcast:31 -> rows 2, 3
#undef CL_SCAN_STEP
      const uint32_t my_e =
          (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(glo & 15u), 0x138, 0xf, 0xf, false);  // wave_shr:1; lane 0: 0
      // walk the true symbols from the entry, compacting them to ent[lane][0..ns)
      if (my_e != 15) {
        uint32_t q = my_e;
        a = a0 + q;
        while (q < kClSlice && a0 + q + 14 <= E) {
          const uint32_t en = C.ent[lane][q];
          C.ent[lane][ns++] = (uint16_t)en;
          q += en >> 12;
        }
        x = a0 + q;
      }
      // slices after the one that stopped at E start (and end) where it stopped
      const uint64_t stopped = __ballot(my_e != 15 && x < stop);
      if (stopped) {
        const uint32_t sl = (uint32_t)__ffsll((unsigned long long)stopped) - 1;
        const uint32_t xs = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)sl);
        if (lane > sl) {
          a = x = xs;
          ns = 0;
        }
      }
    } else {
    auto decode_slice = [&]() {
      x = a;
      ns = 0;
      while (x < stop && x + 14 <= E) {
        const uint32_t b = peek32(W, x);
        const uint32_t e = L.dist[b & 127];
        const uint32_t nb = (e >> 16) & 31, sym = e & 0xffff;
        const uint32_t xb = sym < 16 ? 0u : sym == 16 ? 2u : sym == 17 ? 3u : 7u;
        const uint32_t ext = (b >> nb) & ((1u << xb) - 1);
        if (ns < kClMaxSym) C.ent[lane][ns] = (uint16_t)(sym | (ext << 5) | ((nb + xb) << 12));
        ++ns;
        x += nb + xb;
      }
    };
    decode_slice();
    for (;;) {  // sync: restart each slice from its predecessor's exit
      uint32_t px = __shfl_up(x, 1, 64);
      if (lane == 0) px = a0;
      const bool need = px != a;
      if (__ballot(need) == 0) break;
      if (need) {
        a = px;
        decode_slice();
      }
    }
    }
    // run lengths of this lane's symbols and its last defined value
    uint32_t cnt = 0, own = 0, has = 0;
    for (uint32_t j = 0; j < ns && j < kClMaxSym; ++j) {
      const uint32_t en = C.ent[lane][j], sym = en & 31, ext = (en >> 5) & 127;
      cnt += sym < 16 ? 1u : sym == 18 ? 11u + ext : 3u + ext;
      if (sym != 16) {
        own = sym < 16 ? sym : 0u;
        has = 1;
      }
    }
    const bool bad_lane = ns > kClMaxSym;
    const uint32_t incl = wave_incl_scan_dpp(cnt);  // DPP: no LDS round trips
    const uint32_t base = done + incl - cnt;
    const uint64_t reach = __ballot(done + incl >= ntot);
    const uint32_t lend = reach ? (uint32_t)__ffsll((unsigned long long)reach) - 1 : 63u;
    // value entering each lane (for repeat codes): last defined value before
    // it, as a max-scan of (lane + 1) << 8 | value over the defining lanes
    const uint32_t key = wave_incl_max_dpp(has ? ((lane + 1u) << 8) | own : 0u);
    const uint32_t in_key = __shfl_up(key, 1, 64);
    uint32_t in_v = in_key & 0xffu, in_h = in_key != 0;
    if (lane == 0 || !in_h) {
      in_v = prevv;
      in_h = have_prev;
    }
    // write this lane's runs
    uint32_t i = base, last = in_v, hl = in_h, xe = a;
    bool bad = bad_lane;
    if (lane <= lend) {
      for (uint32_t j = 0; j < ns && j < kClMaxSym && i < ntot; ++j) {
        const uint32_t en = C.ent[lane][j], sym = en & 31, ext = (en >> 5) & 127;
        uint32_t val, rep;
        if (sym < 16) { val = sym; rep = 1; }
        else if (sym == 16) { val = last; rep = 3 + ext; bad |= !hl; }
        else if (sym == 17) { val = 0; rep = 3 + ext; }
        else { val = 0; rep = 11 + ext; }
        if (i + rep > ntot) { bad = true; break; }
        for (uint32_t k = 0; k < rep; ++k) L.lens[i + k] = (uint8_t)val;
        i += rep;
        last = val;
        hl = 1;
        xe += en >> 12;
      }
    }
    if (__ballot(bad)) return DH_TRUNC;
    if (reach) {  // this window completes the header: end = after lane lend's last used symbol
      const uint32_t end = (uint32_t)__builtin_amdgcn_readlane((int)xe, (int)lend);  // lend is wave-uniform
      if (end > E) return DH_TRUNC;
      *end_pos = rfl(end);
      break;
    }
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (tot == 0) return DH_TRUNC;  // no progress (ran past the staged window)
    done += tot;
    const uint32_t k63 = (uint32_t)__builtin_amdgcn_readlane((int)key, 63);
    if (k63) {
      prevv = k63 & 0xffu;
      have_prev = 1;
    }
    p = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  }
  wave_sync();
  if (rfl(L.lens[256]) == 0) return DH_TRUNC;
  if (rfl(build_tab<REG>(L, L.lens, (int)hlit, kLitRoot, 0, L.lit, L.cnt_lit, L.sort_lit, L.litsub, kLitSubCap)))
    return DH_TRUNC;
  if (rfl(build_tab<REG>(L, L.lens + hlit, (int)hdist, kDistRoot, 1, L.dist, L.cnt_dist, L.sort_dist, L.distsub,
                      kDistSubCap)))
    return DH_TRUNC;
  pair_literals(L);
  return DH_OK;
}

// First DEFLATE block of every BGZF block: header + tables built ahead of the
// decode kernel, one wave per block at high occupancy, so the serial header
// work of one block overlaps the others instead of idling a decode workgroup.
// status 0: tables[blockIdx.x] holds the table image and the symbols start at
// bit B0; anything else (stored / fixed block, malformed or long header) is
// left to k_inflate_huff's inline path, which owns the error semantics.
constexpr uint32_t kTabStageBytes = 1024;
// Round 0 parses the header at the start of the block; later rounds the one
// where the previous decode round stopped (hout kHuffPending); blocks with
// nothing pending get status 2.
__global__ __launch_bounds__(64) void k_huff_tables(const uint8_t* __restrict__ file,
                                                    const BlockInfo* __restrict__ blocks, uint32_t b0,
                                                    uint8_t* __restrict__ tables,
                                                    HuffTableInfo* __restrict__ tinfo,
                                                    const HuffOut* __restrict__ hout, uint32_t round) {
  __shared__ __attribute__((aligned(16))) HuffLds L;
  ClLds& C = *reinterpret_cast<ClLds*>(L.lit);  // code-length symbols: done before lit[] is built
  // the staged header bits alias litsub[], which is written only after the
  // code lengths are decoded: 11.3 -> 9.9 KB of LDS, 14 -> 16 waves per CU
  uint4* s_in = reinterpret_cast<uint4*>(L.litsub);
  const uint32_t lane = lane_id();
  const uint32_t bi = b0 + blockIdx.x;
  const BlockInfo blk = blocks[bi];
  HuffTableInfo ti{1u, 0u, 0u, 0u};
  const uint64_t sbyte = blk.coff + 18;
  const uint64_t abase = sbyte & ~15ull;
  uint32_t hbit = 8u * (uint32_t)(sbyte - abase);  // the header, relative to abase
  bool todo = blk.isize != 0;
  if (round > 0) {
    const HuffOut ho = hout[bi];
    todo = todo && ho.status == kHuffPending;
    hbit = ho.resume_bit;
    if (!todo) ti.status = 2u;
  }
  if (todo) {
    // stage 1 KiB from the 16 B unit holding the header
    const uint32_t sb = (hbit >> 3) & ~15u;
    const uint32_t cend = (uint32_t)(blk.coff + blk.csize - abase);  // block end, relative to abase
    const uint32_t nreal = min((cend - sb + 15) >> 4, kTabStageBytes / 16);
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(file + abase + sb);
    for (uint32_t i = lane; i <= nreal; i += 64) s_in[i] = src[i];  // +1 pad chunk (file is padded)
    wave_sync();
    SReader R;
    R.W = reinterpret_cast<const uint32_t*>(s_in);
    const uint32_t Ereal = 8u * ((uint32_t)(sbyte - abase) + (blk.csize - 26)) - 8u * sb;
    const uint32_t E = min(Ereal, 128u * nreal);
    R.seek(hbit - 8u * sb);
    R.fill();
    if (R.pos() + 3 <= E && (((uint32_t)R.buf >> 1) & 3u) == 2u) {
      const uint32_t fin = (uint32_t)R.buf & 1u;
      R.consume(3);
      uint32_t b0pos = 0;
      const uint32_t hp = R.pos();
      const uint32_t h = rfl(peek32(R.W, hp));  // (read before the table build overwrites the staged bits)
      if (dyn_header_par<true>(L, C, R.W, hp, E, &b0pos) == DH_OK) {
        wave_sync();
        const uint32_t est = block_bits_estimate(L.lens, (h & 31) + 257, ((h >> 5) & 31) + 1);
        uint4* __restrict__ dst = reinterpret_cast<uint4*>(tables + (uint64_t)blockIdx.x * kTableImage);
        const uint4* img = reinterpret_cast<const uint4*>(&L);
        for (uint32_t i = lane; i < kTableImage / 16; i += 64) dst[i] = img[i];
        ti = HuffTableInfo{0u, b0pos + 8u * sb, fin, est};
      }
    }
  }
  if (lane == 0) tinfo[blockIdx.x] = ti;
}

// Control block: wave 0 -> workgroup (pass parameters) and back (results).
struct HuffCtl {
  uint32_t act;                 // kActDecode / kActDone
  uint32_t B0, out0, tok0;      // all-lane pass: first symbol bit, output / token position
  uint32_t Bend;                // its region end (pass_end; E for a final block)
  uint32_t fe, fx, ftok, fbytes, m3any;  // its result
  uint32_t xx[kHuffWaves], xe[kHuffWaves];  // exit / event of each wave's last lane
  uint32_t red[2 * kHuffWaves];
};
enum : uint32_t { kActDecode = 1, kActDone = 2 };
constexpr uint32_t kHuffLdsBytes = (sizeof(HuffLds) + 15) & ~15u;
constexpr uint32_t kHuffCtlBytes = (sizeof(HuffCtl) + 15) & ~15u;
constexpr uint32_t kHuffStaticBytes = kHuffLdsBytes + kHuffCtlBytes;
// LDS of a phase-A workgroup (static, kHuffStageMaxLds): the staged block at
// offset 0 (its word addresses need no base add, and the three-word peek fits
// the ds_read2 offsets), then the tables and the control block.
constexpr uint32_t kHuffStageCap = kHuffStageMaxLds - kHuffStaticBytes;
static_assert(kHuffStageCap % 16 == 0 && kHuffStageCap >= 16 * 1024, "phase-A LDS budget");

#ifndef HBAM_HUFF_WAVES_PER_SIMD
#define HBAM_HUFF_WAVES_PER_SIMD 4
#endif
constexpr int kHuffWavesPerSimd = HBAM_HUFF_WAVES_PER_SIMD;  // VGPR cap 128 (no spills); LDS admits 4 staged workgroups per CU
// One decode round of one BGZF block (the body of k_inflate_huff), reading the
// compressed bits from an LDS copy of the block (STAGE) or from HBM/L2.
template <bool STAGE>
__device__ __forceinline__ void huff_block(uint8_t* smem, const uint8_t* __restrict__ file,
                                           const BlockInfo* __restrict__ blocks, uint32_t b0, uint64_t chunk_ustart,
                                           uint32_t* __restrict__ tokens, HuffOut* __restrict__ hout,
                                           const uint8_t* __restrict__ tables, const HuffTableInfo* __restrict__ tinfo,
                                           uint32_t round, uint32_t defer) {
  HuffLds& L = *reinterpret_cast<HuffLds*>(smem + kHuffStageCap);
  HuffCtl& C = *reinterpret_cast<HuffCtl*>(smem + kHuffStageCap + kHuffLdsBytes);
  uint4* s_in = reinterpret_cast<uint4*>(smem);
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t bi = b0 + blockIdx.x;
  const BlockInfo blk = blocks[bi];
  const uint32_t isize = blk.isize;
  if (isize == 0) {  // inflate(buf,off,0) returns 0 without reading: nothing to validate
    if (tid == 0 && round == 0) { hout[bi].ntok = 0; hout[bi].status = kOk; }
    return;
  }
  HuffOut h0{0u, kOk, 0u, 0u};
  if (round > 0) {  // only blocks a previous round left pending
    h0 = hout[bi];
    if (h0.status != kHuffPending) return;
  }
  uint32_t* tok_out = tokens + (blk.ustart - chunk_ustart);
  const uint64_t sbyte = blk.coff + 18;  // cdata start
  const uint64_t abase = sbyte & ~15ull;
  const HuffTableInfo ti = tinfo[blockIdx.x];
  {  // stage the block (+16 B of zero-padded file) and its prebuilt tables in LDS
    // One index space over both copies ([0, nq): block, [nq, nq + nt): table
    // image), kStageBatch 16 B loads in flight per thread before their LDS
    // stores: the copy costs about one memory latency instead of one per
    // loop trip.
    // A later round reads nothing before the bit where the last one stopped,
    // so only the 16 B units from there on are staged.
    const uint32_t nq_all = STAGE ? (uint32_t)((blk.coff + blk.csize - abase + 15) >> 4) + 1 : 0u;
    const uint32_t q0 = round > 0 ? min(h0.resume_bit >> 7, nq_all) : 0u;
    const uint32_t nq = nq_all - q0;
    const uint32_t nt = ti.status == 0 ? kTableImage / 16 : 0u;
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(file + abase) + q0;
    const uint4* __restrict__ tsrc = reinterpret_cast<const uint4*>(tables + (uint64_t)blockIdx.x * kTableImage);
    uint4* sdst = s_in + q0;
    uint4* tdst = reinterpret_cast<uint4*>(&L);
    // global -> LDS without registers (global_load_lds_dwordx4): each wave
    // instruction moves 64 consecutive 16 B units to LDS base + lane x 16, all
    // of a workgroup's copies in flight at once (__syncthreads drains them;
    // phase A 8.52 -> 8.00 ms per C2 pass against register staging with 4-10
    // loads in flight per thread)
    typedef __attribute__((address_space(3))) void* lds_vp;
    typedef __attribute__((address_space(1))) void* gbl_vp;
    const uint32_t wv = tid >> 6, ln = tid & 63;
    for (uint32_t u0 = 64 * wv; u0 < nq; u0 += kHuffThreads)
      if (u0 + ln < nq) __builtin_amdgcn_global_load_lds((gbl_vp)(src + u0 + ln), (lds_vp)(sdst + u0), 16, 0, 0);
    for (uint32_t u0 = 64 * wv; u0 < nt; u0 += kHuffThreads)
      if (u0 + ln < nt) __builtin_amdgcn_global_load_lds((gbl_vp)(tsrc + u0 + ln), (lds_vp)(tdst + u0), 16, 0, 0);
  }
  __syncthreads();
  // compressed bits: the LDS copy, or (unstaged) the file in HBM
  const uint32_t* __restrict__ W =
      STAGE ? reinterpret_cast<const uint32_t*>(s_in) : reinterpret_cast<const uint32_t*>(file + abase);
  const uint32_t E = 8u * ((uint32_t)(sbyte - abase) + (blk.csize - 26));  // end of CDATA (bits from W)

  SReader R;  // wave 0's reader
  R.W = W;
  R.buf = 0;
  R.cnt = R.wd = 0;

  uint32_t outpos = h0.outpos, ntok = h0.ntok;
  bool pending = false;  // stopped before the next DEFLATE block's header (defer)
  uint32_t resume_bit = 0;
  int err = kOk;
  bool look = false;       // output exactly full: zlib's lookahead
  bool final_blk = false;  // BFINAL of the current DEFLATE block
  bool resume = false;     // an all-lane pass result waits in C
  bool pre = ti.status == 0;  // first DEFLATE block's header + tables come from k_huff_tables
  uint32_t est = 0, bend = E;  // wave 0: the current block's size estimate, the pass region end

  // zlib's lookahead once the output is exactly full: decode on until a
  // symbol needs room; returns true when it ends at a (non-final) EOB so the
  // next block header must be examined too.
  auto lookahead = [&]() -> bool {
    for (;;) {
      R.fill();
      const uint32_t p = R.pos();
      const uint32_t e = lit_lookup<true>(L, R.buf);
      const uint32_t n1 = (e >> 16) & 31;
      if (e < kKindLit) return false;  // literal: no room (a pair's first code is checked by n1 >= its length)
      const uint32_t k = e >> 26;
      if (k == K_LEN) {
        const uint32_t ex = (e >> 9) & 15;
        if (p + n1 + ex > E) return false;
        R.consume(n1 + ex);
        R.fill();
        const uint32_t d = dist_lookup<true>(L, R.buf);
        const uint32_t dn = (d >> 16) & 31;
        if (d >= kKindLit) {
          if (R.pos() + max(dn, 1u) <= E) err = kErrIO;
          return false;
        }
        const uint32_t dx = (d >> 21) & 15;
        if (R.pos() + dn + dx > E) return false;
        const uint32_t dist = (d & 0x7fff) + ((uint32_t)(R.buf >> dn) & ((1u << dx) - 1));
        if (dist > outpos) err = kErrIO;
        return false;
      }
      if (k == K_EOB) {
        if (p + n1 > E) return false;
        R.consume(n1);
        return !final_blk;
      }
      if (p + max(n1, 1u) <= E) err = kErrIO;  // invalid literal/length code
      return false;
    }
  };

  if (wave == 0) R.seek(round > 0 ? h0.resume_bit : 8u * (uint32_t)(sbyte - abase));
  for (;;) {
    if (wave == 0) {
      uint32_t act = kActDone;
      for (;;) {  // wave-uniform: advance to the next all-lane pass or to the end
        bool do_look = false;
        if (resume) {  // ---- result of the all-lane pass
          resume = false;
          const uint32_t fe = rfl(C.fe), fxs = rfl(C.fx), m3any = rfl(C.m3any);
          ntok = rfl(ntok + C.ftok);
          outpos = rfl(outpos + C.fbytes);
          if (!m3any && bend < E && fxs < E && outpos < isize) {
            // the pass ended at its region end inside the block: go on with
            // the same tables over the next stretch
            bend = min(E, fxs + (est >> 2) + 4096u);
            if (lane == 0) {
              C.B0 = fxs;
              C.Bend = bend;
              C.out0 = outpos;
              C.tok0 = ntok;
            }
            act = kActDecode;
            resume = true;
            break;
          }
          if (!m3any) {  // walked to the end of CDATA without an end-of-block
            if (outpos < isize) err = kErrFormat;
            else if (outpos == isize) { look = true; R.seek(fxs); }
            else break;
            if (err != kOk || fxs >= E) break;
            do_look = true;
          } else if (fe == EV_EOB) {
            R.seek(fxs);
            if (final_blk) { err = kErrFormat; break; }  // EOB before ISIZE bytes
            if (defer) {  // the next header is the next round's (k_huff_tables)
              pending = true;
              resume_bit = fxs;
              break;
            }
            continue;
          } else if (fe == EV_FULLX) {
            look = true;
            R.seek(fxs);
            do_look = true;
          } else if (fe == EV_FULLO) {
            break;
          } else {
            err = fe == EV_ERR ? kErrIO : kErrFormat;
            break;
          }
        } else if (pre) {  // ---- first DEFLATE block: prebuilt tables already in LDS
          pre = false;
          final_blk = ti.final_blk != 0;
          R.seek(ti.B0);
          est = ti.est_bits;
          bend = pass_end(ti.B0, est, final_blk, E);
          if (lane == 0) {
            C.B0 = ti.B0;
            C.Bend = bend;
            C.out0 = outpos;
            C.tok0 = ntok;
          }
          act = kActDecode;
          resume = true;
          break;
        } else {  // ---- next DEFLATE block header
          if (err != kOk) break;
          R.fill();
          if (R.pos() + 3 > E) { if (!look) err = kErrFormat; break; }
          const uint32_t hdr = (uint32_t)R.buf & 7;
          R.consume(3);
          final_blk = hdr & 1;
          const uint32_t type = hdr >> 1;
          if (type == 0) {  // stored
            R.consume((8u - (R.pos() & 7u)) & 7u);  // to the byte boundary
            R.fill();
            if (R.pos() + 32 > E) { if (!look) err = kErrFormat; break; }
            const uint32_t len = (uint32_t)R.buf & 0xffff, nlen = (uint32_t)(R.buf >> 16) & 0xffff;
            R.consume(32);
            if (len != (~nlen & 0xffffu)) { err = kErrIO; break; }
            const uint32_t p = R.pos();  // byte aligned
            if (look) {
              if (len != 0) break;  // COPY with no room: zlib stops here
              if (final_blk) break;
              continue;
            }
            const uint32_t n = min(min(len, isize - outpos), (E - p) >> 3);
            const uint8_t* src = reinterpret_cast<const uint8_t*>(W) + (p >> 3);
            for (uint32_t j = lane; j < n; j += 64) tok_out[ntok + j] = (1u << 24) | src[j];
            ntok += n;
            outpos += n;
            R.seek(p + 8 * n);
            if (n < len) {
              if (outpos < isize) err = kErrFormat;  // ran out of input
              break;
            }
            if (final_blk) {
              if (outpos < isize) err = kErrFormat;
              break;
            }
            if (outpos == isize) look = true;
            continue;
          }
          if (type == 3) { err = kErrIO; break; }
          const uint32_t hp = R.pos();
          if (type == 1) {  // fixed Huffman
            for (int s = lane; s < 320; s += 64) {
              uint8_t l;
              if (s < 144) l = 8; else if (s < 256) l = 9; else if (s < 280) l = 7; else if (s < 288) l = 8; else l = 5;
              L.lens[s] = l;
            }
            wave_sync();
            if (rfl(build_table(L, L.lens, 288, kLitRoot, 0, L.lit, L.cnt_lit, L.sort_lit, L.litsub, kLitSubCap)) ||
                rfl(build_table(L, L.lens + 288, 32, kDistRoot, 1, L.dist, L.cnt_dist, L.sort_dist, L.distsub,
                                kDistSubCap))) {
              err = kErrIO;
              break;
            }
            pair_literals(L);
            est = block_bits_estimate(L.lens, 288, 32);
          } else {  // dynamic Huffman: code lengths decoded by the 64 lanes of the wave
            uint32_t endp = 0;
            int dh = dyn_header_par<false>(L, *reinterpret_cast<ClLds*>(L.lit), W, R.pos(), E, &endp);
            if (rfl(dh) == DH_OK) {
              R.seek(endp);
            } else {  // an anomaly: the serial parse owns zlib's error semantics
              dh = dyn_header(L, R, E);
              if (dh == DH_TRUNC) { if (!look) err = kErrFormat; break; }
              if (dh != DH_OK) { err = kErrIO; break; }
            }
            const uint32_t h = rfl(peek32(W, hp));
            est = block_bits_estimate(L.lens, (h & 31) + 257, ((h >> 5) & 31) + 1);
          }
          if (!look) {  // hand the symbol stream to the workgroup
            bend = pass_end(R.pos(), est, final_blk, E);
            if (lane == 0) {
              C.Bend = bend;
              C.B0 = R.pos();
              C.out0 = outpos;
              C.tok0 = ntok;
            }
            act = kActDecode;
            resume = true;
            break;
          }
          do_look = true;
        }
        if (do_look) {
          if (!lookahead()) break;
        }
      }
      if (lane == 0) C.act = act;
    }
    __syncthreads();
    if (C.act != kActDecode) break;

    // ---- all-lane decode of this DEFLATE block's symbols
    const uint32_t B0 = C.B0, out0 = C.out0, tok0 = C.tok0, Bend = C.Bend;
    const uint32_t R = Bend > B0 ? Bend - B0 : 0u;
    const uint32_t S = (R + kHuffThreads - 1) / kHuffThreads;
    uint32_t a = min(B0 + tid * S, Bend);
    const uint32_t stop = tid == kHuffThreads - 1 ? Bend : min(B0 + (tid + 1) * S, Bend);
    MergePts mp;
    uint32_t mj = 0, x, nt, nb;
    const uint32_t mf = S < kMergeTinyBits ? kMergeFirst / 4 : S < kMergeShortBits ? kMergeFirst / 2 : kMergeFirst;
    uint32_t ev = lane_decode<LD_SPEC>(L, W, a, stop, E, x, nt, nb, mp, mj, nullptr, 0, 0, mf);
    const uint32_t sx = x, snt = nt, snb = nb, sev = ev;
    for (;;) {  // sync: restart each slice from its predecessor's exit
      if (lane == 63) {
        C.xx[wave] = x;
        C.xe[wave] = ev;
      }
      __syncthreads();
      uint32_t px = __shfl_up(x, 1, 64), pev = __shfl_up(ev, 1, 64);
      if (lane == 0 && wave > 0) {
        px = C.xx[wave - 1];
        pev = C.xe[wave - 1];
      }
      const bool need = tid > 0 && pev == EV_STOP && px != a;
      if (!wg_any(need, C.red)) break;
      if (need) {
        a = px;
        uint32_t rx, rnt, rnb;
        const uint32_t rev = lane_decode<LD_SYNC>(L, W, a, stop, E, rx, rnt, rnb, mp, mj, nullptr, 0, 0, mf);
        if (rev == EV_MERGE) {  // shares the speculative walk from boundary mj on
          const uint32_t bj = mj == 0 ? mp.b0 : mj == 1 ? mp.b1 : mj == 2 ? mp.b2 : mp.b3;
          x = sx;
          ev = sev;
          nt = rnt + snt - (mf << mj);
          nb = rnb + snb - bj;
        } else {
          x = rx;
          ev = rev;
          nt = rnt;
          nb = rnb;
        }
      }
    }
    const uint32_t lend0 = wg_min(ev != EV_STOP ? tid : 0xffffffffu, C.red);
    const uint32_t lend = lend0 == 0xffffffffu ? (uint32_t)kHuffThreads - 1 : lend0;
    const bool valid = tid <= lend;
    uint32_t toff, boff;
    wg_excl_scan2(valid ? nt : 0u, valid ? nb : 0u, C.red, toff, boff);
    uint32_t x3 = a, nt3 = 0, nb3 = 0, ev3 = EV_STOP;
    if (valid)
      ev3 = lane_decode<LD_EMIT>(L, W, a, stop, E, x3, nt3, nb3, mp, mj, tok_out + tok0 + toff, out0 + boff, isize);
    const uint32_t m3 = wg_min((valid && ev3 != EV_STOP) ? tid : 0xffffffffu, C.red);
    const uint32_t f = m3 != 0xffffffffu ? m3 : lend;
    if (tid == f) {
      C.fe = ev3;
      C.fx = x3;
      C.ftok = toff + nt3;
      C.fbytes = boff + nb3;
      C.m3any = m3 != 0xffffffffu;
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (wave == 0 && pending && err == kOk) {
      hout[bi] = HuffOut{ntok, kHuffPending, resume_bit, outpos};
    } else {
      if (err == kOk && outpos < isize) err = kErrFormat;  // "Did not inflate expected amount"
      hout[bi] = HuffOut{ntok, err, 0u, outpos};
    }
  }
}

// Phase A: one 256-thread workgroup per BGZF block of the chunk.  Each
// workgroup stages its compressed block in LDS when it fits kHuffStageCap,
// else it reads the bits from HBM/L2: one launch per round whatever the block
// sizes (a launch used to run unstaged as a whole when one block of the chunk
// was too big).
__global__ __launch_bounds__(kHuffThreads, kHuffWavesPerSimd) void k_inflate_huff(
    const uint8_t* __restrict__ file, const BlockInfo* __restrict__ blocks, uint32_t b0, uint64_t chunk_ustart,
    uint32_t* __restrict__ tokens, HuffOut* __restrict__ hout, const uint8_t* __restrict__ tables,
    const HuffTableInfo* __restrict__ tinfo, uint32_t round, uint32_t defer) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kHuffStageCap + kHuffStaticBytes];
  const BlockInfo& b = blocks[b0 + blockIdx.x];
  const uint64_t abase = (b.coff + 18) & ~15ull;
  const uint32_t need = (uint32_t)(((b.coff + b.csize - abase + 15) >> 4) + 1) * 16u;  // huff_stage_bytes
  if (need <= kHuffStageCap)
    huff_block<true>(smem, file, blocks, b0, chunk_ustart, tokens, hout, tables, tinfo, round, defer);
  else
    huff_block<false>(smem, file, blocks, b0, chunk_ustart, tokens, hout, tables, tinfo, round, defer);
}

// ---------------------------------------------------------------------------
// Inflate phase B: tokens -> bytes, one 1024-thread workgroup per BGZF block
// ---------------------------------------------------------------------------
// Every output position p gets a u16 entry in an LDS map: 0xFF00|byte for a
// literal, else the position its byte is copied from (p - dist, strictly
// smaller; for an overlapping match this is the periodic extension, so every
// match is expanded in one parallel step).  Bytes are then resolved by
// following entries back to a literal and writing the result in place (path
// compression); positions are visited in increasing order so chains are
// short (measured on BAM data: mean depth 7.5, max ~40 without compression).
// The map needs ISIZE <= 65280 (positions below the 0xFF00 tag space: the
// BGZF maximum htsjdk/bgzip write); larger blocks take the dependency-round
// path over a byte image in the same LDS.
constexpr int kLzThreads = 1024;
constexpr int kLzWaves = kLzThreads / 64;
constexpr uint32_t kMapMax = 65280;
constexpr uint32_t kLitTag = 0xFF00u;
// map entries: 128 KiB, so that the 16 waves' 8 rows of 64 eight-entry chunks
// (step 3) cover it exactly and need no bounds (o0 + ISIZE <= 65295)
constexpr uint32_t kMapEntries = 65536;
static_assert(kMapEntries == kLzWaves * 8 * 64 * 8 && kMapMax + 15 < kMapEntries, "phase-B map geometry");
constexpr int kLzRing = 4;  // phase-B fill: 64-token groups loaded ahead (4 vs 8 measured equal)
constexpr int kLzTokGroups = 32;  // token groups a wave keeps in registers (32 K tokens per block)
#ifndef HBAM_LZ_CHASE
#define HBAM_LZ_CHASE 2
#endif
constexpr int kLzChase = HBAM_LZ_CHASE;  // positions chased together per thread (4: slower before pointer jumping)

// exclusive scan over the workgroup; returns the prefix, *total = sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) scratch[wid] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kLzWaves; ++w) {
    const uint32_t x = scratch[w];
    off += (uint32_t)w < wid ? x : 0u;
    tot += x;
  }
  *total = tot;
  __syncthreads();
  return off + inc - v;
}

__device__ __forceinline__ uint32_t block_min(uint32_t v, uint32_t* scratch) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d, 64));
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  uint32_t r = 0xffffffffu;
#pragma unroll
  for (int w = 0; w < kLzWaves; ++w) r = min(r, scratch[w]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint32_t tok_len(uint32_t t) { return (t >> 31) ? (t & 0xffffu) : ((t >> 24) & 3u); }

// Rare path (ISIZE > 65280): byte image, matches resolve in dependency rounds.
__device__ void lz77_rounds(uint8_t* out, uint32_t* scratch, const uint32_t* tk, uint32_t ntok, uint32_t isize,
                            uint32_t o0) {
  uint32_t P = 0;
  for (uint32_t c = 0; c < ntok; c += kLzThreads) {
    const uint32_t i = c + threadIdx.x;
    const uint32_t t = i < ntok ? tk[i] : 0u;
    const bool ismatch = (t >> 31) != 0;
    const uint32_t len = i < ntok ? tok_len(t) : 0u;
    uint32_t total;
    const uint32_t pos = P + block_excl_scan(len, scratch, &total);
    P += total;
    if (!ismatch) {
      for (uint32_t j = 0; j < len; ++j)
        if (pos + j < isize) out[o0 + pos + j] = (uint8_t)(t >> (8 * j));
    }
    const uint32_t dist = ((t >> 16) & 0x7fffu) + 1;
    bool pending = ismatch && pos < isize;
    __syncthreads();
    for (;;) {
      const uint32_t first = block_min(pending ? pos : 0xffffffffu, scratch);
      if (first == 0xffffffffu) break;
      if (pending && (pos == first || pos - dist + min(len, dist) <= first)) {
        const uint32_t n = min(len, isize - pos);
        uint8_t* dst = out + o0 + pos;
        for (uint32_t k = 0; k < n; ++k) dst[k] = dst[(int)k - (int)dist];
        pending = false;
      }
      __syncthreads();
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kLzThreads) void k_inflate_lz77(const BlockInfo* __restrict__ blocks, uint32_t b0,
                                                             uint64_t chunk_ustart,
                                                             const uint32_t* __restrict__ tokens,
                                                             const HuffOut* __restrict__ hout,
                                                             uint8_t* __restrict__ u) {
  // map index = o0 + position, so 16-byte output segments read 32 B-aligned LDS
  __shared__ __attribute__((aligned(16))) uint16_t map[kMapEntries];
  __shared__ uint32_t scratch[kLzWaves];
  const BlockInfo blk = blocks[b0 + blockIdx.x];
  const HuffOut ho = hout[b0 + blockIdx.x];
  if (ho.status != kOk || blk.isize == 0) return;
  const uint32_t isize = blk.isize;
  const uint32_t o0 = (uint32_t)(blk.ustart & 15);
  const uint32_t* tk = tokens + (blk.ustart - chunk_ustart);
  const uint32_t ntok = ho.ntok;
  const uint32_t tid = threadIdx.x;
  const uint64_t g0 = blk.ustart & ~15ull;
  const uint64_t gend = blk.ustart + isize;
  const uint32_t nseg = (uint32_t)((gend - g0 + 15) >> 4);

  if (isize > kMapMax) {  // uniform per workgroup
    uint8_t* img = reinterpret_cast<uint8_t*>(map);
    lz77_rounds(img, scratch, tk, ntok, isize, o0);
    for (uint32_t s = tid; s < nseg; s += kLzThreads) {
      const uint64_t ga = g0 + 16ull * s;
      if (ga >= blk.ustart && ga + 16 <= gend) {
        *reinterpret_cast<uint4*>(u + ga) = *reinterpret_cast<const uint4*>(img + 16 * s);
      } else {
        for (int j = 0; j < 16; ++j) {
          const uint64_t g = ga + j;
          if (g >= blk.ustart && g < gend) u[g] = img[16 * s + j];
        }
      }
    }
    return;
  }

  // 1. wave w expands tokens [w*TW, (w+1)*TW); its output range starts at
  //    the byte total of the waves before it.  Up to kLzTokGroups groups of
  //    64 tokens stay in registers from this load to step 2 (all loads in
  //    flight at once); a wave with more re-reads them (L2) through a ring.
  const uint32_t wid = tid >> 6, lane = tid & 63;
  // 0. empty map: 0 marks a position no token writes (inside a match)
  auto zero_map = [&]() {
    for (uint32_t c = tid; c < kMapEntries / 8; c += kLzThreads)
      reinterpret_cast<uint4*>(map)[c] = make_uint4(0u, 0u, 0u, 0u);
  };
  const uint32_t TW = (ntok + kLzWaves - 1) / kLzWaves;
  const uint32_t tw0 = min(wid * TW, ntok), tw1 = min(tw0 + TW, ntok);
  const bool inreg = TW <= 64u * kLzTokGroups;  // uniform over the workgroup
  uint32_t tr[kLzTokGroups];
  uint32_t wsum = 0;
  if (inreg) {
#pragma unroll
    for (int k = 0; k < kLzTokGroups; ++k) {
      const uint32_t i = tw0 + lane + 64u * k;
      tr[k] = i < tw1 ? tk[i] : 0u;  // 0 = a literal token of length 0
    }
    zero_map();  // (while the loads are in flight)
#pragma unroll
    for (int k = 0; k < kLzTokGroups; ++k) wsum += tok_len(tr[k]);
  } else {
    zero_map();
    for (uint32_t i0 = tw0 + lane; i0 < tw1 + lane; i0 += 8 * 64) {  // 8 loads in flight
      uint32_t tv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) tv[k] = i0 + 64 * k < tw1 ? tk[i0 + 64 * k] : 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) wsum += tok_len(tv[k]);
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) wsum += __shfl_xor(wsum, d, 64);
  if (lane == 0) scratch[wid] = wsum;
  __syncthreads();
  uint32_t P = 0;
#pragma unroll
  for (int w = 0; w < kLzWaves; ++w) P += (uint32_t)w < wid ? scratch[w] : 0u;
  const uint32_t whi = min(P + wsum, isize);  // end of this wave's range (the last token may run past ISIZE)

  // 2. token heads, 64 tokens (one per lane) at a time: a literal writes its
  //    1-2 entries (tag | byte), a match only its distance at its first
  //    position.  Every lane stores at most two entries, whatever the
  //    match lengths of its wave.
  uint16_t* m = map + o0;
  auto head = [&](uint32_t t) {
    const uint32_t len = tok_len(t);
    const uint32_t incl = wave_incl_scan_dpp(len);
    const uint32_t pos = P + incl - len;
    P += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (len != 0 && pos < whi) {
      if (t >> 31) {
        m[pos] = (uint16_t)(((t >> 16) & 0x7fffu) + 1);  // dist <= pos: checked in phase A
      } else {
        m[pos] = (uint16_t)(kLitTag | (t & 0xffu));
        if (len == 2 && pos + 1 < whi) m[pos + 1] = (uint16_t)(kLitTag | ((t >> 8) & 0xffu));
      }
    }
  };
  // one token's entries, branch-free selects and two predicated stores
  auto head_at = [&](uint32_t t, uint32_t len, uint32_t pos) {
    const bool mt = (t >> 31) != 0;
    const uint32_t e0 = mt ? ((t >> 16) & 0x7fffu) + 1u : (kLitTag | (t & 0xffu));  // dist <= pos: checked in phase A
    if ((len != 0) & (pos < whi)) m[pos] = (uint16_t)e0;
    if ((len == 2) & !mt & (pos + 1 < whi)) m[pos + 1] = (uint16_t)(kLitTag | ((t >> 8) & 0xffu));
  };
  if (inreg) {
    // two groups of 64 tokens per scan: their lengths packed in 16-bit
    // halves (a group's bytes <= 64 x 258 < 2^16)
#pragma unroll
    for (int j = 0; j < kLzTokGroups / 2; ++j) {
      if (tw0 + 128u * j >= tw1) break;  // wave-uniform
      const uint32_t t0 = tr[2 * j], t1 = tr[2 * j + 1];
      const uint32_t l0 = tok_len(t0), l1 = tok_len(t1);
      const uint32_t incl = wave_incl_scan_dpp(l0 | (l1 << 16));
      const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      const uint32_t p0 = P + (incl & 0xffffu) - l0;
      const uint32_t p1 = P + (tot & 0xffffu) + (incl >> 16) - l1;
      P += (tot & 0xffffu) + (tot >> 16);
      head_at(t0, l0, p0);
      head_at(t1, l1, p1);
    }
  } else {
    uint32_t ring[kLzRing];  // tokens of the next kLzRing groups (L2 hits after step 1)
#pragma unroll
    for (int k = 0; k < kLzRing; ++k) ring[k] = tw0 + lane + 64 * k < tw1 ? tk[tw0 + lane + 64 * k] : 0u;
    for (uint32_t gi = tw0; gi < tw1 && P < whi; gi += 64) {  // wave-uniform
      const uint32_t i = gi + lane;
      const uint32_t t = ring[0];
#pragma unroll
      for (int k = 0; k + 1 < kLzRing; ++k) ring[k] = ring[k + 1];
      ring[kLzRing - 1] = i + 64 * kLzRing < tw1 ? tk[i + 64 * kLzRing] : 0u;
      head(i < tw1 ? t : 0u);
    }
  }
  __syncthreads();

  // 3. match bodies: every 0 entry belongs to the match whose distance is the
  //    nearest non-zero entry before it that is not a literal, so a
  //    carry-forward over the map turns distances into source positions
  //    (q - dist).  Wave w owns 8-entry chunks [512w, 512w + 512), eight
  //    coalesced rows of 64 chunks held in registers.  The carry is a running
  //    max of keys (chunk + 1) << 16 | last non-zero entry of the chunk:
  //    keys grow with the position, so max-scans over rows, lanes (DPP) and
  //    waves (LDS) find the nearest non-zero entry before each chunk.
  {
    constexpr uint32_t kRowChunks = 64, kWaveChunks = 8 * kRowChunks;
    uint4* mc = reinterpret_cast<uint4*>(map);
    uint4 rows[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t c = wid * kWaveChunks + r * kRowChunks + lane;
      rows[r] = mc[c];  // (every chunk: entries past the block are zero or unused)
    }
    uint32_t key[8], kmax = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t w4[4] = {rows[r].x, rows[r].y, rows[r].z, rows[r].w};
      uint32_t rl = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rl = (w4[j] & 0xffffu) ? (w4[j] & 0xffffu) : rl;
        rl = (w4[j] >> 16) ? (w4[j] >> 16) : rl;
      }
      const uint32_t c = wid * kWaveChunks + r * kRowChunks + lane;
      key[r] = rl ? ((c + 1u) << 16) | rl : 0u;
      kmax = max(kmax, key[r]);
    }
    const uint32_t wmax = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_dpp(kmax), 63);
    if (lane == 0) scratch[wid] = wmax;
    __syncthreads();
    uint32_t carry = 0;  // key of the last non-zero entry before this wave's chunks
    for (uint32_t w = 0; w < wid; ++w) carry = max(carry, scratch[w]);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t incl = wave_incl_max_dpp(key[r]);
      const uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xf, 0xf, true);  // wave_shr:1
      uint32_t cur = max(carry, excl) & 0xffffu;
      carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, 63));
      const uint32_t c = wid * kWaveChunks + r * kRowChunks + lane;
      // position of entry 0 of this chunk, relative to the block (index - o0)
      const uint32_t q0 = 8u * c - o0;
      uint32_t w4[4] = {rows[r].x, rows[r].y, rows[r].z, rows[r].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // inside the block a 0 entry follows its match's head, so a literal
        // stays and every other entry (a head's distance, or 0 in its body)
        // becomes q - cur, cur = the last non-zero entry (past the block the
        // values are unused)
        const uint32_t lo = w4[j] & 0xffffu, hi = w4[j] >> 16;
        cur = lo ? lo : cur;
        const uint32_t olo = lo < kLitTag ? q0 + 2u * j - cur : lo;
        cur = hi ? hi : cur;
        const uint32_t ohi = hi < kLitTag ? q0 + 2u * j + 1u - cur : hi;
        w4[j] = (olo & 0xffffu) | (ohi << 16);
      }
      mc[c] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
  __syncthreads();

  // 4. resolve, increasing positions first; results written back in place
  //    (path compression).  Each chase step is one dependent LDS load, so a
  //    thread chases kLzChase positions 1024 apart at once (their loads
  //    overlap).  Any visiting order is correct: entries always point to
  //    smaller positions and a chase ends at a literal, resolved or not.
  // Branch-free steps: a resolved lane re-reads its own entry (no select,
  // no exec-masked read).
  for (uint32_t q = tid; q < isize; q += kLzChase * kLzThreads) {
    uint32_t v[kLzChase], at[kLzChase];
#pragma unroll
    for (int k = 0; k < kLzChase; ++k) {
      at[k] = q + k * kLzThreads < isize ? q + k * kLzThreads : q;
      v[k] = m[at[k]];
    }
    for (;;) {
      bool more = false;
#pragma unroll
      for (int k = 0; k < kLzChase; ++k) more |= v[k] < kLitTag;
      if (!__builtin_amdgcn_ballot_w64(more)) break;
      // min(v, at): an unresolved v is a smaller position than at; a
      // resolved lane (v >= kLitTag > at) re-reads its own entry, which
      // holds v (the literal it first read, or its last store below: only
      // this lane writes m[at]) -- so the value read is the new v either way
#pragma unroll
      for (int k = 0; k < kLzChase; ++k) v[k] = m[min(v[k], at[k])];
      // pointer jumping: every step stores how far the chase got, so a lane
      // whose chain runs through this position skips the hops already made
      // (a run of dist-1 matches resolves in ~log2(len) steps instead of
      // len).  Any stored value is a position holding the same byte, or the
      // byte itself, so racing stores keep every entry valid.  The last step
      // of a chase stores its byte, so nothing is written after the loop.
      // Every lane stores, branch-free (exec-masked stores of only the lanes
      // still chasing: 5.70 vs 5.43 ms per C2 pass).
#pragma unroll
      for (int k = 0; k < kLzChase; ++k) m[at[k]] = (uint16_t)v[k];
    }
  }
  __syncthreads();

  // 5. 16 B stores; low bytes of 16 entries packed with v_perm
  for (uint32_t s = tid; s < nseg; s += kLzThreads) {
    const uint64_t ga = g0 + 16ull * s;
    if (ga >= blk.ustart && ga + 16 <= gend) {
      const uint4 e0 = *reinterpret_cast<const uint4*>(map + 16 * s);
      const uint4 e1 = *reinterpret_cast<const uint4*>(map + 16 * s + 8);
      uint4 o;
      o.x = __builtin_amdgcn_perm(e0.y, e0.x, 0x06040200u);
      o.y = __builtin_amdgcn_perm(e0.w, e0.z, 0x06040200u);
      o.z = __builtin_amdgcn_perm(e1.y, e1.x, 0x06040200u);
      o.w = __builtin_amdgcn_perm(e1.w, e1.z, 0x06040200u);
      *reinterpret_cast<uint4*>(u + ga) = o;
    } else {
      for (int j = 0; j < 16; ++j) {
        const uint64_t g = ga + j;
        if (g >= blk.ustart && g < gend) u[g] = (uint8_t)map[16 * s + j];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Record chain
// ---------------------------------------------------------------------------
struct ChainEnv {
  const uint8_t* u;        // inflated stream
  const BlockInfo* blocks;
  uint64_t e_inf;          // end of inflated (available) data
  uint64_t e_true;         // end of the logical stream (all blocks)
  uint64_t p0;             // span start position (first record, read after seek)
  uint64_t q_end;          // records with position >= q_end are outside the span
  const uint64_t* dead;    // sorted dead positions (empty block after exhausted one)
  uint32_t ndead;
  int32_t n_ref;
  uint32_t k0, k1;         // block range [k0, k1)
  int validate;            // reader mode: 0 SILENT (none), 1 LENIENT (decode structure), 2 STRICT (SAMRecord.isValid)
  const int32_t* ref_len;  // n_ref reference lengths, or nullptr
};

// ---------------------------------------------------------------------------
// [htsjdk] SAMRecord.isValid under ValidationStringency.STRICT.  BAMFileReader's
// iterator validates every record it returns unless the stringency is SILENT
// (BAMRecordReader.java:142,192-194 pass hadoopbam.samheaderreader.
// validation-stringency through; htsjdk's default is STRICT) and STRICT turns
// the first error into a SAMFormatException.  Restated subset (DESIGN.md
// §2.1; oracle/hbam_oracle.c orc_strict_invalid is the same rule list):
//   structure  read name, cigar, seq, qual inside the record; cigar op <= 8
//   unpaired   no proper-pair / mate-unmapped / mate-reverse / first / second
//              flag, mate refID == -1
//   paired     mate refID/pos consistent (isValidReferenceIndexAndPosition),
//              mate refID set unless mate-unmapped, first or second flag
//   unmapped   not secondary / supplementary, MAPQ 0, no cigar
//   mapped     cigar present, non-empty sequence dictionary
//   position   refID/pos consistent, pos+1 <= reference length
//   cigar      Cigar.isValid (zero-length ops, H/S/P placement, I/D pairs,
//              a real operator) and M/=/X blocks inside the reference
//   bin        == reg2bin(alignmentStart-1, alignmentEnd)
//   seq        cigar read length == l_seq when both are non-zero;
//              l_seq == 0 needs FZ, or CQ + CS (unless secondary)
// The reader's IllegalArgumentException (refID out of range) is checked
// before this, as the record factory raises it first.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int reg2bin_dev(int beg, int end) {  // GenomicIndexUtil.regionToBin
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

// aux tag t present (an l_seq == 0 record's FZ / CQ / CS lookup); *zlen = Z
// string length
__device__ bool aux_find(const uint8_t* u, uint64_t a, uint64_t e, uint16_t tag, int64_t* zlen) {
  while (a + 3 <= e) {
    const uint16_t t = (uint16_t)(u[a] | (u[a + 1] << 8));
    const uint8_t ty = u[a + 2];
    a += 3;
    int64_t sz;
    switch (ty) {
      case 'A': case 'c': case 'C': sz = 1; break;
      case 's': case 'S': sz = 2; break;
      case 'i': case 'I': case 'f': sz = 4; break;
      case 'Z': case 'H': {
        uint64_t j = a;
        while (j < e && u[j]) ++j;
        if (t == tag) *zlen = (int64_t)(j - a);
        sz = (int64_t)(j - a) + 1;
        break;
      }
      case 'B': {
        if (a + 5 > e) return false;
        const uint8_t sub = u[a];
        const int32_t cnt = (int32_t)ldu32(u, a + 1);
        const int es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
        if (cnt < 0) return false;
        sz = 5 + (int64_t)cnt * es;
        break;
      }
      default: return false;
    }
    if (t == tag) return true;
    if ((uint64_t)sz > e - a) return false;  // a malformed aux block ends the lookup
    a += (uint64_t)sz;
  }
  return false;
}

// true when the (fully inflated) record at q fails validation.  strict =
// false keeps only the structural decode failures (LENIENT still decodes the
// cigar for isValid and logs the rest).
// *defer (when given): a cigar longer than kWaveCigarOps operators is not
// checked here (false returned, *defer set) -- record_invalid_wave takes it.
constexpr uint32_t kWaveCigarOps = 32;
// (h: the record's head, load_head(E.u, q), already in registers)
__device__ __forceinline__ bool record_invalid_h(const ChainEnv& E, uint64_t q, int32_t bs, bool strict, bool* defer,
                                                 const RecHead& h) {
  const uint8_t* u = E.u;
  const int32_t ref = (int32_t)h.at(1), pos = (int32_t)h.at(2);
  const uint32_t w12 = h.at(3), w16 = h.at(4);
  const uint32_t lrn = w12 & 0xffu, mapq = (w12 >> 8) & 0xffu, bin = w12 >> 16;
  const uint32_t ncig = w16 & 0xffffu, flag = w16 >> 16;
  if (defer && ncig > kWaveCigarOps) {
    *defer = true;
    return false;
  }
  const int32_t lseq = (int32_t)h.at(5), nref = (int32_t)h.at(6), npos = (int32_t)h.at(7);
  // structure: the lazy fields isValid decodes must lie inside the record
  if (lrn < 1 || lseq < 0) return true;
  const int64_t need = 32 + (int64_t)lrn + 4 * (int64_t)ncig + ((int64_t)lseq + 1) / 2 + (int64_t)lseq;
  if (need > (int64_t)bs) return true;
  const uint64_t c0 = q + 36 + lrn;
  uint32_t qlen = 0, rlen = 0;
  for (uint32_t k = 0; k < ncig; ++k) {
    const uint32_t op = ldu32(u, c0 + 4ull * k) & 0xfu;
    if (op > 8) return true;
  }
  if (!strict) return false;
  const bool paired = flag & 0x1, unmapped = flag & 0x4;
  if (!paired) {
    if (flag & (0x2 | 0x8 | 0x20 | 0x40 | 0x80)) return true;
    if (nref != -1) return true;
  } else {
    if (nref == -1) {
      if (npos != -1) return true;
      if (!(flag & 0x8)) return true;  // "Mapped mate should have mate reference name"
    } else {
      if (npos == -1) return true;
      if (E.ref_len && (int64_t)npos + 1 > (int64_t)E.ref_len[nref]) return true;
    }
    if (!(flag & 0xC0)) return true;  // neither first nor second of pair
  }
  if (unmapped) {
    if (flag & (0x100 | 0x800)) return true;
    if (mapq != 0) return true;  // (a cigar on an unmapped read is allowed: test.bam has them)
  } else {
    if (ncig == 0) return true;
    if (E.n_ref == 0) return true;  // MISSING_SEQUENCE_DICTIONARY
  }
  if (ref == -1) {
    if (pos != -1) return true;
  } else {
    if (pos == -1) return true;
    if (E.ref_len && (int64_t)pos + 1 > (int64_t)E.ref_len[ref]) return true;
  }
  // cigar: Cigar.isValid + alignment blocks (mapped reads only)
  bool real = false;
  int64_t rpos = (int64_t)pos + 1, maxend = 0;
  uint32_t prev_op = 99, first_op = 99, last_op = 99;
  if (ncig) {
    first_op = ldu32(u, c0) & 0xfu;
    last_op = ldu32(u, c0 + 4ull * (ncig - 1)) & 0xfu;
  }
  // Cigar.isValid: between two separators (M/=/X/N or P) an I or a D may
  // appear only once ("No M or N operator between pair of I/D operators")
  bool seen_i = false, seen_d = false;
  for (uint32_t k = 0; k < ncig; ++k) {
    const uint32_t c = ldu32(u, c0 + 4ull * k), op = c & 0xfu, len = c >> 4;
    const bool consumes_read = op == 0 || op == 1 || op == 4 || op == 7 || op == 8;
    const bool consumes_ref = op == 0 || op == 2 || op == 3 || op == 7 || op == 8;
    if (consumes_read) qlen += len;
    if (consumes_ref) rlen += len;
    if (!unmapped) {
      if (len == 0) return true;
      if (op == 5) {
        if (k != 0 && k != ncig - 1) return true;
      } else if (op == 4) {
        if (k == 0 || k == ncig - 1) {
        } else if (k == 1) {
          if (!(ncig == 3 && last_op == 5) && first_op != 5) return true;
        } else if (k == ncig - 2) {
          if (last_op != 5) return true;
        } else {
          return true;
        }
      } else if (op == 6) {
        if (k != 0) {
          if (k == ncig - 1) return true;
          const uint32_t nx = ldu32(u, c0 + 4ull * (k + 1)) & 0xfu;
          const bool pr = prev_op <= 3 || prev_op == 7 || prev_op == 8, nr = nx <= 3 || nx == 7 || nx == 8;
          if (!pr || !nr) return true;
        }
        seen_i = seen_d = false;
      } else {  // real operator
        real = true;
        if (op == 1) {
          if (seen_i) return true;
          seen_i = true;
        } else if (op == 2) {
          if (seen_d) return true;
          seen_d = true;
        } else {
          seen_i = seen_d = false;
        }
        if (op == 0 || op == 7 || op == 8) maxend = max(maxend, rpos + (int64_t)len - 1);
      }
    }
    if (consumes_ref) rpos += len;
    prev_op = op;
  }
  if (!unmapped) {
    if (!real) return true;
    if (ref >= 0 && E.ref_len && maxend > (int64_t)E.ref_len[ref]) return true;  // CIGAR_MAPS_OFF_REFERENCE
  }
  // bin: computeIndexingBin()
  {
    const int start0 = pos;  // getAlignmentStart() - 1
    int end = unmapped ? 0 : (int)((int64_t)pos + 1 + (int64_t)rlen - 1);
    if (end <= 0) end = start0 + 1;
    if ((uint32_t)reg2bin_dev(start0, end) != bin) return true;
  }
  if (lseq != 0 && ncig != 0 && (int64_t)qlen != (int64_t)lseq) return true;  // MISMATCH_CIGAR_SEQ_LENGTH
  if (lseq == 0 && !(flag & 0x100)) {  // EMPTY_READ unless FZ, or CQ and CS
    const uint64_t a0 = c0 + 4ull * ncig, ae = q + 4 + (uint64_t)bs;
    int64_t zl = -1;
    if (!aux_find(u, a0, ae, (uint16_t)('F' | ('Z' << 8)), &zl)) {
      int64_t cq = -1, cs = -1;
      const bool hq = aux_find(u, a0, ae, (uint16_t)('C' | ('Q' << 8)), &cq);
      const bool hs = aux_find(u, a0, ae, (uint16_t)('C' | ('S' << 8)), &cs);
      if (!hq || !hs || cq <= 0 || cs <= 0) return true;
    }
  }
  return false;
}

__device__ bool record_invalid(const ChainEnv& E, uint64_t q, int32_t bs, bool strict, bool* defer = nullptr) {
  return record_invalid_h(E, q, bs, strict, defer, load_head(E.u, q));
}

// record_invalid by a whole wave, for records with long cigars (ONT-like
// reads carry thousands of operators; one lane walking them serially set the
// pace of the record check: 2.0 ms per C4 pass).  Same rules, same result: the
// per-operator rules become a lane-per-operator pass over chunks of 64, the
// running state becomes scans --
//   qlen / rlen            wrapping u32 sums (as the serial u32 accumulators)
//   alignment block ends   exclusive 64-bit sum of reference lengths before k
//   Cigar.isValid I/D pairs   an I (D) is invalid when the previous I (D)
//                          comes after the last separator (M N = X P) before it:
//                          two running max-scans of 1-based indices.
// Wave-uniform arguments; returns the same value on every lane.
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
    if (lane >= (uint32_t)d) v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)(uint64_t)v, d, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v >> 32), d, 64);
    v = max(v, (int64_t)(((uint64_t)hi << 32) | lo));
  }
  return v;
}

__device__ bool record_invalid_wave(const ChainEnv& E, uint64_t q, int32_t bs, bool strict) {
  const uint8_t* u = E.u;
  const uint32_t lane = lane_id();
  const int32_t ref = (int32_t)ldu32(u, q + 4), pos = (int32_t)ldu32(u, q + 8);
  const uint32_t w12 = ldu32(u, q + 12), w16 = ldu32(u, q + 16);
  const uint32_t lrn = w12 & 0xffu, mapq = (w12 >> 8) & 0xffu, bin = w12 >> 16;
  const uint32_t ncig = w16 & 0xffffu, flag = w16 >> 16;
  const int32_t lseq = (int32_t)ldu32(u, q + 20), nref = (int32_t)ldu32(u, q + 24), npos = (int32_t)ldu32(u, q + 28);
  if (lrn < 1 || lseq < 0) return true;
  const int64_t need = 32 + (int64_t)lrn + 4 * (int64_t)ncig + ((int64_t)lseq + 1) / 2 + (int64_t)lseq;
  if (need > (int64_t)bs) return true;
  const uint64_t c0 = q + 36 + lrn;
  bool bad = false;
  for (uint32_t k = lane; k < ncig; k += 64) bad |= (ldu32(u, c0 + 4ull * k) & 0xfu) > 8;
  if (__ballot(bad)) return true;
  if (!strict) return false;
  const bool paired = flag & 0x1, unmapped = flag & 0x4;
  if (!paired) {
    if (flag & (0x2 | 0x8 | 0x20 | 0x40 | 0x80)) return true;
    if (nref != -1) return true;
  } else {
    if (nref == -1) {
      if (npos != -1) return true;
      if (!(flag & 0x8)) return true;
    } else {
      if (npos == -1) return true;
      if (E.ref_len && (int64_t)npos + 1 > (int64_t)E.ref_len[nref]) return true;
    }
    if (!(flag & 0xC0)) return true;
  }
  if (unmapped) {
    if (flag & (0x100 | 0x800)) return true;
    if (mapq != 0) return true;
  } else {
    if (ncig == 0) return true;
    if (E.n_ref == 0) return true;
  }
  if (ref == -1) {
    if (pos != -1) return true;
  } else {
    if (pos == -1) return true;
    if (E.ref_len && (int64_t)pos + 1 > (int64_t)E.ref_len[ref]) return true;
  }
  const uint32_t first_op = ncig ? ldu32(u, c0) & 0xfu : 99u;
  const uint32_t last_op = ncig ? ldu32(u, c0 + 4ull * (ncig - 1)) & 0xfu : 99u;
  uint32_t qlen = 0, rlen = 0;          // lane partial sums (wrapping, as the serial code)
  uint64_t rcarry = 0;                  // reference bases of the chunks before
  uint32_t sep_carry = 0, i_carry = 0, d_carry = 0;  // 1-based indices of the last separator / I / D
  bool real = false;
  int64_t maxend = 0;
  for (uint32_t k0 = 0; k0 < ncig; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool in = k < ncig;
    const uint32_t c = in ? ldu32(u, c0 + 4ull * k) : 0u, op = in ? c & 0xfu : 15u, len = c >> 4;
    const bool consumes_read = op == 0 || op == 1 || op == 4 || op == 7 || op == 8;
    const bool consumes_ref = op == 0 || op == 2 || op == 3 || op == 7 || op == 8;
    if (consumes_read) qlen += len;
    if (consumes_ref) rlen += len;
    const uint64_t rl = consumes_ref ? (uint64_t)len : 0ull;
    const uint64_t rincl = wave_incl_sum64(rl);
    const int64_t rpos = (int64_t)pos + 1 + (int64_t)(rcarry + rincl - rl);  // before op k
    rcarry += (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)rincl, 63) |
              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rincl >> 32), 63) << 32);
    // running 1-based indices (0 = none) up to and including op k
    const bool sep = op == 0 || op == 3 || op == 6 || op == 7 || op == 8;
    const uint32_t sep_i = max(sep_carry, wave_incl_max_dpp(sep ? k + 1 : 0u));
    const uint32_t i_i = max(i_carry, wave_incl_max_dpp(op == 1 ? k + 1 : 0u));
    const uint32_t d_i = max(d_carry, wave_incl_max_dpp(op == 2 ? k + 1 : 0u));
    // the same before op k (exclusive): one lane up, the carry on lane 0
    uint32_t sep_x = (uint32_t)__shfl_up((int)sep_i, 1, 64), i_x = (uint32_t)__shfl_up((int)i_i, 1, 64),
             d_x = (uint32_t)__shfl_up((int)d_i, 1, 64);
    if (lane == 0) {
      sep_x = sep_carry;
      i_x = i_carry;
      d_x = d_carry;
    }
    sep_carry = (uint32_t)__builtin_amdgcn_readlane((int)sep_i, 63);
    i_carry = (uint32_t)__builtin_amdgcn_readlane((int)i_i, 63);
    d_carry = (uint32_t)__builtin_amdgcn_readlane((int)d_i, 63);
    if (in && !unmapped) {
      if (len == 0) bad = true;
      if (op == 5) {
        if (k != 0 && k != ncig - 1) bad = true;
      } else if (op == 4) {
        if (k == 0 || k == ncig - 1) {
        } else if (k == 1) {
          if (!(ncig == 3 && last_op == 5) && first_op != 5) bad = true;
        } else if (k == ncig - 2) {
          if (last_op != 5) bad = true;
        } else {
          bad = true;
        }
      } else if (op == 6) {
        if (k != 0) {
          if (k == ncig - 1) {
            bad = true;
          } else {
            const uint32_t pv = ldu32(u, c0 + 4ull * (k - 1)) & 0xfu, nx = ldu32(u, c0 + 4ull * (k + 1)) & 0xfu;
            const bool pr = pv <= 3 || pv == 7 || pv == 8, nr = nx <= 3 || nx == 7 || nx == 8;
            if (!pr || !nr) bad = true;
          }
        }
      } else {  // real operator
        real = true;
        if (op == 1 && i_x > sep_x) bad = true;  // a second I since the last separator
        if (op == 2 && d_x > sep_x) bad = true;
        if (op == 0 || op == 7 || op == 8) maxend = max(maxend, rpos + (int64_t)len - 1);
      }
    }
  }
  if (__ballot(bad)) return true;
  qlen = wave_sum_u32(qlen);
  rlen = wave_sum_u32(rlen);
  if (!unmapped) {
    if (__ballot(real) == 0) return true;
    maxend = wave_max_i64(maxend);
    if (ref >= 0 && E.ref_len && maxend > (int64_t)E.ref_len[ref]) return true;
  }
  {
    const int start0 = pos;
    int end = unmapped ? 0 : (int)((int64_t)pos + 1 + (int64_t)rlen - 1);
    if (end <= 0) end = start0 + 1;
    if ((uint32_t)reg2bin_dev(start0, end) != bin) return true;
  }
  if (lseq != 0 && ncig != 0 && (int64_t)qlen != (int64_t)lseq) return true;
  if (lseq == 0 && !(flag & 0x100)) {
    const uint64_t a0 = c0 + 4ull * ncig, ae = q + 4 + (uint64_t)bs;
    int64_t zl = -1;
    if (!aux_find(u, a0, ae, (uint16_t)('F' | ('Z' << 8)), &zl)) {
      int64_t cq = -1, cs = -1;
      const bool hq = aux_find(u, a0, ae, (uint16_t)('C' | ('Q' << 8)), &cq);
      const bool hs = aux_find(u, a0, ae, (uint16_t)('C' | ('S' << 8)), &cs);
      if (!hq || !hs || cq <= 0 || cs <= 0) return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool is_dead(const ChainEnv& E, uint64_t q) {
  uint32_t lo = 0, hi = E.ndead;  // sorted; usually 0 or 1 entries (the EOF marker)
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (E.dead[mid] < q) lo = mid + 1; else hi = mid;
  }
  return lo < E.ndead && E.dead[lo] == q;
}
__device__ __forceinline__ bool dead_in_record(const ChainEnv& E, uint64_t q, int32_t bs) {
  if (E.ndead == 0) return false;
  const uint8_t offs[11] = {4, 8, 12, 13, 14, 16, 18, 20, 24, 28, 32};
  for (int i = 0; i < 11; ++i)
    if (is_dead(E, q + offs[i])) return true;
  return bs > 32 && is_dead(E, q + 36);
}

// Is any dead position within [q, q + 40] (header fields + first rest byte)?
__device__ __forceinline__ bool dead_near(const ChainEnv& E, uint64_t q) {
  uint32_t lo = 0, hi = E.ndead;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (E.dead[mid] < q) lo = mid + 1; else hi = mid;
  }
  return lo < E.ndead && E.dead[lo] <= q + 40;
}

// Necessary conditions for a record of a well-formed BAM (guess only; the
// true chain is fixed by the link step, never by this test).  Bytes past the
// inflated range of a stream that goes on (an open window, or blocks not yet
// inflated) cannot refute a record: it stays plausible when its block_size
// can be read and is >= 32 (so a walk through it still moves forward).
// (Taken as implausible, the record straddling a window's end within its
// first 36 + l_read_name bytes failed every candidate walk of its block, and
// the block's search walked from every later candidate: ~7 ms on one 256 MiB
// drop-in window.)
__device__ __forceinline__ bool plausible(const ChainEnv& E, uint64_t q) {
  if (q + 36 > E.e_inf) return E.e_inf < E.e_true && q + 4 <= E.e_inf && (int32_t)ldu32(E.u, q) >= 32;
  const RecHead h = load_head(E.u, q);
  int32_t bs = (int32_t)h.at(0);
  int32_t ref = (int32_t)h.at(1);
  int32_t pos = (int32_t)h.at(2);
  uint32_t lrn = h.at(3) & 0xffu;
  uint32_t ncig = h.at(4) & 0xffffu;
  int32_t lseq = (int32_t)h.at(5);
  int32_t nref = (int32_t)h.at(6);
  int32_t npos = (int32_t)h.at(7);
  if (ref < -1 || ref >= E.n_ref || nref < -1 || nref >= E.n_ref) return false;
  if (pos < -1 || npos < -1 || lrn < 1 || lseq < 0) return false;
  int64_t need = 32 + (int64_t)lrn + 4 * (int64_t)ncig + (int64_t)lseq + ((int64_t)lseq + 1) / 2;
  if ((int64_t)bs < need) return false;
  if (q + 4 + (uint64_t)bs > E.e_true) return false;
  if (q + 36 + lrn > E.e_inf) return E.e_inf < E.e_true;
  return E.u[q + 36 + lrn - 1] == 0;
}

// plausible() split for a software-pipelined walk: plausible_head decides
// from q's head h alone (1: plausible, 0: not, 2: the read-name end byte at
// q + 36 + lrn - 1 decides: *name_at = its position), so that a walk can
// load that byte together with the next record's head (q + 4 + block_size):
// one dependent memory round trip per record instead of two.  Same result
// as plausible(E, q) when h = load_head(E.u, q).
__device__ __forceinline__ int plausible_head(const ChainEnv& E, uint64_t q, const RecHead& h, uint64_t* name_at) {
  if (q + 36 > E.e_inf) return E.e_inf < E.e_true && q + 4 <= E.e_inf && (int32_t)h.at(0) >= 32;
  int32_t bs = (int32_t)h.at(0);
  int32_t ref = (int32_t)h.at(1);
  int32_t pos = (int32_t)h.at(2);
  uint32_t lrn = h.at(3) & 0xffu;
  uint32_t ncig = h.at(4) & 0xffffu;
  int32_t lseq = (int32_t)h.at(5);
  int32_t nref = (int32_t)h.at(6);
  int32_t npos = (int32_t)h.at(7);
  if (ref < -1 || ref >= E.n_ref || nref < -1 || nref >= E.n_ref) return 0;
  if (pos < -1 || npos < -1 || lrn < 1 || lseq < 0) return 0;
  int64_t need = 32 + (int64_t)lrn + 4 * (int64_t)ncig + (int64_t)lseq + ((int64_t)lseq + 1) / 2;
  if ((int64_t)bs < need) return 0;
  if (q + 4 + (uint64_t)bs > E.e_true) return 0;
  if (q + 36 + lrn > E.e_inf) return E.e_inf < E.e_true;
  *name_at = q + 36 + lrn - 1;
  return 2;
}

// plausible() at q and at the record after it (or the end / unreadable data):
// a cheap second check that removes most false candidates inside long records.
__device__ __forceinline__ bool plausible2(const ChainEnv& E, uint64_t q) {
  if (!plausible(E, q)) return false;
  const uint64_t q2 = q + 4 + (uint64_t)(int32_t)ldu32(E.u, q);
  return q2 == E.e_true || q2 + 36 > E.e_inf || plausible(E, q2);
}

// A necessary condition of plausible() that reads 8 bytes: refID and mate
// refID in range (random bytes pass with probability ~(n_ref / 2^32)^2), or
// data past the inflated range, which plausible() judges itself.  Candidate
// scans test it first and run plausible2 only when a lane of the wave passes.
__device__ __forceinline__ bool cand_prefilter(const ChainEnv& E, uint64_t q) {
  if (q + 36 > E.e_inf) return true;
  const int32_t ref = (int32_t)ldu32(E.u, q + 4), nref = (int32_t)ldu32(E.u, q + 24);
  return ref >= -1 && ref < E.n_ref && nref >= -1 && nref < E.n_ref;
}

// One chain step from q under the given rules.  Returns false if the walk
// cannot continue (data unavailable or malformed record); *nq = next position.
template <int MODE>
__device__ __forceinline__ bool chain_step(const ChainEnv& E, uint64_t q, uint64_t* nq) {
  if (q + 4 > E.e_inf) return false;
  int32_t bs = (int32_t)ldu32(E.u, q);
  if (MODE == kReader) {
    if (bs < 32) return false;
    *nq = q + 4 + (uint64_t)bs;
  } else {
    *nq = q + 4 + (bs > 0 ? (uint64_t)bs : 0);
  }
  return true;
}

// Link the per-block guesses into the true chain (serial in block order, with
// a 256-block tile fast path when every block of the tile links to the next).
// entry[i] = true first record position of block k0+i, or kNone.
// summary[0] = final chain position, summary[1] = 1 if the chain stopped
// inside a block (malformed record / data unavailable).
template <int MODE>
__global__ __launch_bounds__(256) void k_rec_link(ChainEnv E, const uint64_t* __restrict__ g,
                                                  const uint64_t* __restrict__ x, uint64_t* __restrict__ entry,
                                                  uint64_t* __restrict__ summary) {
  __shared__ uint64_t s_cur;
  __shared__ int s_stop;
  const uint32_t nb = E.k1 - E.k0;
  if (threadIdx.x == 0) { s_cur = E.p0; s_stop = 0; }
  __syncthreads();
  for (uint32_t t0 = 0; t0 < nb; t0 += 256) {
    const uint32_t i = t0 + threadIdx.x;
    const uint64_t cur = s_cur;
    const int stop = s_stop;
    bool fast = true;
    if (i < nb) {
      const BlockInfo b = E.blocks[E.k0 + i];
      const uint64_t bend = b.ustart + b.isize;
      const uint64_t gi = g[i], xi = x[i];
      const uint64_t expect = (threadIdx.x == 0) ? cur : x[i - 1];
      fast = !stop && gi != kNone && gi == expect && gi < E.q_end && xi != kNone && xi >= bend;
    }
    const int all_fast = __syncthreads_and(fast);
    if (all_fast) {
      if (i < nb) entry[i] = g[i];
      __syncthreads();
      if (threadIdx.x == 0) s_cur = x[min(t0 + 255, nb - 1)];
      __syncthreads();
      continue;
    }
    if (threadIdx.x == 0) {
      uint64_t c = cur;
      int st = stop;
      for (uint32_t j = t0; j < min(t0 + 256, nb); ++j) {
        const BlockInfo b = E.blocks[E.k0 + j];
        const uint64_t bend = b.ustart + b.isize;
        if (st || c >= E.q_end || c >= bend || b.isize == 0) {
          entry[j] = kNone;
          continue;
        }
        entry[j] = c;
        if (g[j] == c) {
          c = x[j];
        } else {
          uint64_t q = c, nq;
          while (q < bend && chain_step<MODE>(E, q, &nq)) q = nq;
          c = q;
        }
        if (c < bend) st = 1;
      }
      s_cur = c;
      s_stop = st;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    summary[0] = s_cur;
    summary[1] = (uint64_t)s_stop;
  }
}

// Parallel link.  y[i] = guess exit of block i (0 when the block has no
// guess); in[i] = max(y[0..i-1]) is the position the chain enters block i
// with, IF every guess is on the true chain.  k_rec_link_check verifies that
// claim block by block (entry = guess where the chain enters the block,
// pass-through elsewhere) and counts violations; any violation sends the span
// to the exact serial link (k_rec_link).
__global__ void k_rec_link_y(const uint64_t* __restrict__ g, const uint64_t* __restrict__ x, uint32_t nb,
                             uint64_t* __restrict__ y) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) y[i] = (g[i] != kNone && x[i] != kNone) ? x[i] : 0;
}

// Count (and validate) the records of each block of the span under the
// reader / indexer rules.  One thread per block.
//   cnt[i], err[i] = status code, errpos[i] = position of the failing record,
//   *need = furthest byte the span needs inflated (atomicMax).
template <int MODE>
__global__ void k_rec_count(ChainEnv E, const uint64_t* __restrict__ entry, uint32_t* __restrict__ cnt,
                            int32_t* __restrict__ err, unsigned long long* __restrict__ need) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nb = E.k1 - E.k0;
  if (i >= nb) return;
  uint32_t n = 0;
  int st = kOk;
  const uint64_t e = entry[i];
  if (e != kNone) {
    const BlockInfo b = E.blocks[E.k0 + i];
    const uint64_t lim = min(b.ustart + b.isize, E.q_end);
    uint64_t q = e;
    bool first = (MODE == kReader) && (e == E.p0);  // reader: first record follows a seek
    while (q < lim) {
      if (!first && is_dead(E, q)) {  // readInt at an exhausted block + empty block: EOF
        st = kStopClean;
        break;
      }
      first = false;
      const uint64_t avail = E.e_true - q;
      if (avail < 4) {
        st = MODE == kIndexer && avail > 0 ? kErrIO : kStopClean;  // "less than 4 bytes long" / EOF
        break;
      }
      if (q + 4 > E.e_inf) { atomicMax(need, (unsigned long long)(q + 4)); break; }
      const int32_t bs = (int32_t)ldu32(E.u, q);
      if (MODE == kReader) {
        if (bs < 32) { st = kErrFormat; break; }
        if (dead_in_record(E, q, bs) || avail - 4 < (uint64_t)bs) { st = kErrTrunc; break; }
        if (q + 4 + (uint64_t)bs > E.e_inf) { atomicMax(need, (unsigned long long)(q + 4 + (uint64_t)bs)); break; }
        const int32_t ref = (int32_t)ldu32(E.u, q + 4), nref = (int32_t)ldu32(E.u, q + 24);
        if (ref < -1 || ref >= E.n_ref || nref < -1 || nref >= E.n_ref) { st = kErrArg; break; }
        if (E.validate && record_invalid(E, q, bs, E.validate == 2)) { st = kErrFormat; break; }
        ++n;
        q += 4 + (uint64_t)bs;
      } else {
        ++n;
        if (bs > 0) {
          if ((uint64_t)bs > avail - 4 || is_dead(E, q + 4)) { st = kErrIO; break; }  // "Skip failed"
          q += 4 + (uint64_t)bs;
        } else {
          q += 4;
        }
      }
    }
  }
  cnt[i] = n;
  err[i] = st;
}

// Second walk: write record positions and normalized voffs at base[i].
template <int MODE>
__global__ void k_rec_emit(ChainEnv E, const uint64_t* __restrict__ entry, const uint32_t* __restrict__ cnt,
                           const uint64_t* __restrict__ base, uint64_t* __restrict__ rec_pos,
                           uint64_t* __restrict__ rec_voff) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nb = E.k1 - E.k0;
  if (i >= nb) return;
  const uint32_t n = cnt[i];
  if (n == 0) return;
  const BlockInfo b = E.blocks[E.k0 + i];
  uint64_t q = entry[i];
  uint64_t o = base[i];
  for (uint32_t r = 0; r < n; ++r) {
    rec_pos[o + r] = q;
    rec_voff[o + r] = (b.coff << 16) | (q - b.ustart);
    const int32_t bs = (int32_t)ldu32(E.u, q);
    q += 4 + (uint64_t)(MODE == kReader ? bs : (bs > 0 ? bs : 0));
  }
}

// ---------------------------------------------------------------------------
// Fused record decode: SoA columns + BAMRecordReader.getKey
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// MurmurHash3.murmurhash3(byte[], seed) (util/MurmurHash3.java:32-102) over
// len bytes of u at off.
__device__ uint64_t murmur3_dev(const uint8_t* u, uint64_t off, uint32_t len, int32_t seed) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = (uint64_t)(int64_t)seed, h2 = h1;
  const uint32_t nblocks = len / 16;
  for (uint32_t i = 0; i < nblocks; ++i) {
    uint64_t k1 = ldu64(u, off + 16ull * i), k2 = ldu64(u, off + 16ull * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = (h2 << 31) | (h1 >> 33); h2 += h1; h2 = h2 * 5 + 0x38495ab5;  // :59
  }
  const uint64_t t = off + 16ull * nblocks;
  const uint32_t r = len & 15;
  if (r) {
    // tail bytes via two 8-byte loads (padding makes the over-read safe), masked
    uint64_t lo = ldu64(u, t), hi = ldu64(u, t + 8);
    if (r > 8) {
      uint64_t k2 = hi & (~0ull >> (64 - 8 * (r - 8)));
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    uint64_t k1 = r >= 8 ? lo : (lo & (~0ull >> (64 - 8 * r)));
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)len;
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// Fields + key of the record at q into slot i of the columns.
__device__ __forceinline__ void decode_record_h(const uint8_t* __restrict__ u, uint64_t q, uint64_t i,
                                                const Columns& col, const RecHead& h) {
  const int32_t bs = (int32_t)h.at(0);
  const int32_t ref = (int32_t)h.at(1);
  const int32_t pos = (int32_t)h.at(2);
  const uint32_t w12 = h.at(3);
  const uint32_t w16 = h.at(4);
  const int32_t lseq = (int32_t)h.at(5);
  const int32_t nref = (int32_t)h.at(6);
  const int32_t npos = (int32_t)h.at(7);
  const int32_t tlen = (int32_t)h.at(8);
  const uint16_t flag = (uint16_t)(w16 >> 16);
  col.ref_id[i] = ref;
  col.pos[i] = pos;
  col.l_read_name[i] = (uint8_t)w12;
  col.mapq[i] = (uint8_t)(w12 >> 8);
  col.bin[i] = (uint16_t)(w12 >> 16);
  col.n_cigar[i] = (uint16_t)w16;
  col.flag[i] = flag;
  col.l_seq[i] = lseq;
  col.next_ref_id[i] = nref;
  col.next_pos[i] = npos;
  col.tlen[i] = tlen;
  col.rest_off[i] = q + 36;
  col.rest_len[i] = (uint32_t)(bs - 32);
  // BAMRecordReader.getKey (:81-121): alignmentStart = pos+1
  const int32_t start = (int32_t)((uint32_t)pos + 1u);
  int64_t key;
  if (!((flag & 4) || ref < 0 || start < 0)) {
    key = (int64_t)(((uint64_t)(int64_t)ref << 32) | (uint64_t)(int64_t)(int32_t)(start - 1));
  } else {
    if (col.long_rec && (uint32_t)(bs - 32) > kLongHash) {  // long rest: k_long_hash
      const uint32_t slot = atomicAdd(col.long_n, 1u);
      if (slot < col.long_cap) {
        col.long_rec[slot] = i;
        return;
      }
    }
    const int32_t mh = (int32_t)murmur3_dev(u, q + 36, (uint32_t)(bs - 32), 0);
    key = (int64_t)((0x7fffffffull << 32) | (uint64_t)(int64_t)mh);
  }
  col.key[i] = key;
}
__device__ __forceinline__ void decode_record(const uint8_t* __restrict__ u, uint64_t q, uint64_t i,
                                              const Columns& col) {
  decode_record_h(u, q, i, col, load_head(u, q));
}

// Murmur keys of long unmapped records (C4-like reads: the rest is tens of
// KB), one wave per record.  The per-block input mixing (k1*c1, rotl, *c2 and
// the k2 twin) is independent across 16 B blocks, so the 64 lanes do it for
// 64 consecutive blocks from one coalesced 1 KB load; only the h1/h2 chain is
// serial, and it runs on wave-uniform values (scalar ALU) fed by readlane.
// A speculative launch (queued before the host has read k_rec_check_out's
// verdict) passes a gate: it runs only if no block stopped the span
// (*bad == ~0) and no record needs bytes past the inflated range; otherwise
// rec_pos past the stop may be stale and the host launches it again.
struct SpecGate {
  const unsigned long long* bad = nullptr;  // nullptr: no gate
  const unsigned long long* need = nullptr;
  uint64_t e_inf = 0;
};
__device__ __forceinline__ bool gate_closed(const SpecGate& g) {
  return g.bad && (*g.bad != ~0ull || *g.need > g.e_inf);
}
__global__ __launch_bounds__(64) void k_long_hash(const uint8_t* __restrict__ u, const uint64_t* __restrict__ rec_pos,
                                                  Columns col, SpecGate gate) {
  if (gate_closed(gate)) return;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  const uint32_t lane = lane_id();
  const uint32_t nrec = min(*col.long_n, col.long_cap);
  for (uint32_t li = blockIdx.x; li < nrec; li += gridDim.x) {
    const uint64_t i = col.long_rec[li];
    const uint64_t q = rec_pos[i];
    const uint32_t len = ldu32(u, q) - 32u;
    const uint64_t off = q + 36;
    uint64_t h1 = 0, h2 = 0;  // seed 0 (BAMRecordReader.java:101)
    const uint32_t nblocks = len / 16;
    // the next 64 blocks are loaded while the serial chain runs over these
    uint64_t n1 = 0, n2 = 0;
    if (lane < nblocks) {
      n1 = ldu64(u, off + 16ull * lane);
      n2 = ldu64(u, off + 16ull * lane + 8);
    }
    for (uint32_t c = 0; c < nblocks; c += 64) {
      uint64_t k1 = n1, k2 = n2;
      const uint32_t nb = c + 64 + lane;
      n1 = n2 = 0;
      if (nb < nblocks) {
        n1 = ldu64(u, off + 16ull * nb);
        n2 = ldu64(u, off + 16ull * nb + 8);
      }
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2;
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1;
      const uint32_t k1lo = (uint32_t)k1, k1hi = (uint32_t)(k1 >> 32);
      const uint32_t k2lo = (uint32_t)k2, k2hi = (uint32_t)(k2 >> 32);
      const uint32_t m = min(64u, nblocks - c);
      for (uint32_t j = 0; j < m; ++j) {  // util/MurmurHash3.java:48-60, :59 quirk
        const uint64_t K1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)k1hi, (int)j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)k1lo, (int)j);
        const uint64_t K2 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)k2hi, (int)j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)k2lo, (int)j);
        h1 ^= K1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        h2 ^= K2;
        h2 = (h2 << 31) | (h1 >> 33); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
      }
    }
    const uint64_t t = off + 16ull * nblocks;
    const uint32_t r = len & 15;
    if (r) {  // tail (:62-88), as murmur3_dev
      const uint64_t lo = ldu64(u, t), hi = ldu64(u, t + 8);
      if (r > 8) {
        uint64_t k2 = hi & (~0ull >> (64 - 8 * (r - 8)));
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      }
      uint64_t k1 = r >= 8 ? lo : (lo & (~0ull >> (64 - 8 * r)));
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len;
    h2 ^= (uint64_t)len;
    h1 += h2;
    h2 += h1;
    h1 = fmix64(h1);
    h2 = fmix64(h2);
    h1 += h2;
    if (lane == 0) col.key[i] = (int64_t)((0x7fffffffull << 32) | (uint64_t)(int64_t)(int32_t)h1);
  }
}

__global__ void k_rec_decode(const uint8_t* __restrict__ u, const uint64_t* __restrict__ rec_pos, uint64_t n,
                             Columns col) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    decode_record(u, rec_pos[i], i, col);
}

// ---------------------------------------------------------------------------
// Record chain v2: lane-per-block walks with per-block record lists
// ---------------------------------------------------------------------------
//   k_rec_cand     one wave per block: first plausible record start (512
//                  positions per step) -- where the block's guess walk begins.
//   k_rec_walk     one lane per block: the chain from that candidate (next
//                  candidates on failure), from the span start, or from a
//                  forced (true) entry; every record start of the block is
//                  listed as a u16 offset.  All walks of a span are in flight
//                  at once, so the span costs one dependent-load chain of
//                  ~records-per-block steps instead of a wave per block.
//   k_rec_linkfix  max-scan link check; blocks whose list is off the chain are
//                  re-walked from their true entry (usually zero or a few).
//   k_rec_check_out  one wave per block: the reader / indexer rules of
//                  k_rec_count for every listed record at once (the first stop
//                  gives count, status and the bytes still to inflate), then
//                  positions, voffs and (reader) the fused decode + key at the
//                  block's scanned base.
// k_rec_cand: one wave per block, each lane testing kCandPos consecutive
// positions per step (512 per step): refID and mate refID of its 8 positions
// come from 5 aligned 8 B loads, and only the rare position that passes that
// test runs plausible2; the first hit wins (ballot).  A short-read block
// finishes in its first step, at the cost of the old 64-positions step; a
// long-read block (C4: the first record start lies ~32 KB in on average)
// takes 8x fewer dependent steps (0.74 ms per C4 pass before).
constexpr int kCandPos = 8;
template <int MODE>
__global__ __launch_bounds__(64) void k_rec_cand(ChainEnv E, uint64_t* __restrict__ cand) {
  const uint32_t k = E.k0 + blockIdx.x;
  const BlockInfo b = E.blocks[k];
  const uint64_t bend = b.ustart + b.isize;
  const uint32_t lane = lane_id();
  uint64_t c = kNone;
  if (bend > E.p0 && b.ustart > E.p0 && b.ustart < E.q_end && b.isize > 0) {
    const uint64_t s0 = b.ustart & ~7ull;  // 8-aligned scan origin (positions < ustart are masked)
    for (uint64_t c0 = s0; c0 < bend; c0 += 64 * kCandPos) {
      const uint64_t p0 = c0 + (uint64_t)lane * kCandPos;
      uint32_t pass = 0;  // bit j: position p0 + j passes the prefilter
      if (p0 < bend) {
        uint32_t w[10];
        const uint2* src = reinterpret_cast<const uint2*>(E.u + p0);  // du_ is padded past the stream
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const uint2 v = src[i];
          w[2 * i] = v.x;
          w[2 * i + 1] = v.y;
        }
#pragma unroll
        for (int j = 0; j < kCandPos; ++j) {
          const uint64_t q = p0 + j;
          const int32_t ref = (int32_t)__builtin_amdgcn_alignbyte(w[2 + (j >> 2)], w[1 + (j >> 2)], j & 3);
          const int32_t nref = (int32_t)__builtin_amdgcn_alignbyte(w[7 + (j >> 2)], w[6 + (j >> 2)], j & 3);
          const bool ok = q >= b.ustart && q < bend &&
                          (q + 36 > E.e_inf || (ref >= -1 && ref < E.n_ref && nref >= -1 && nref < E.n_ref));
          pass |= ok ? 1u << j : 0u;
        }
      }
      uint32_t hit = kCandPos;  // the first position of this lane that is plausible2
      if (__ballot(pass != 0)) {
        for (uint32_t m = pass; m; m &= m - 1) {
          const uint32_t j = (uint32_t)__ffs((int)m) - 1;
          if (plausible2(E, p0 + j)) {
            hit = j;
            break;
          }
        }
      }
      const uint64_t hm = __ballot(hit < kCandPos);
      if (hm) {
        const uint32_t f = (uint32_t)__ffsll((long long)hm) - 1;
        c = c0 + (uint64_t)f * kCandPos + (uint32_t)__shfl((int)hit, (int)f, 64);
        break;
      }
    }
    // A start 1-3 bytes before a true record reads that record's block_size
    // shifted up by whole bytes (~2^8-2^24 times it) and, with refID 0, its
    // fields stay in range: plausible2 passes and the walk leaves the block
    // at once -- past the inflated end of a window it cannot be checked, and
    // the link check then re-walks the block and the ones its far exit hid
    // (one round each; C2 passes took two, drop-in windows fell back to the
    // serial link).  When c's record leaves the block, a plausible2 start
    // 1-3 bytes later whose record ends inside the block is taken instead.
    if (c != kNone && lane == 0 && c + 4 + (uint64_t)(int32_t)ldu32(E.u, c) >= bend) {
      for (uint32_t d = 1; d <= 3; ++d) {
        const uint64_t q = c + d;
        if (q + 36 <= E.e_inf && q + 4 + (uint64_t)(int32_t)ldu32(E.u, q) < bend && plausible2(E, q)) {
          c = q;
          break;
        }
      }
    }
  }
  if (lane == 0) cand[blockIdx.x] = c;
}

constexpr int kGuessLookahead = 4;  // plausible records required past a guess walk's exit
constexpr uint64_t kRetry = ~0ull - 2;  // g[]: the candidate's walk failed, search on
constexpr uint32_t kListPlausible = 0x80000000u;  // wcnt flag: the list came from a plausible() walk
constexpr uint32_t kListCountMask = 0x7fffffffu;

template <int MODE>
__global__ __launch_bounds__(256) void k_rec_walk(ChainEnv E, const uint64_t* __restrict__ cand,
                                                  const uint64_t* __restrict__ force, uint64_t* __restrict__ g_out,
                                                  uint64_t* __restrict__ x_out, uint32_t* __restrict__ wcnt,
                                                  uint16_t* __restrict__ list, uint32_t* __restrict__ overflow,
                                                  bool validate) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nb = E.k1 - E.k0;
  if (force) {
    // A re-walk round forces a few blocks; each is one lane's chain of ~190
    // dependent loads from HBM.  The whole wave first pulls every forced
    // block of the wave (+ the lookahead past its end) into L2 with
    // independent loads, so the chain then runs at L2 latency.
    const uint64_t fi = i < nb ? force[i] : kNone;
    uint64_t todo = __ballot(fi != kNone && fi != kForceEmpty);
    uint32_t acc = 0;
    const uint32_t lane = lane_id();
    while (todo) {
      const uint32_t src = (uint32_t)__ffsll((long long)todo) - 1;
      todo &= todo - 1;
      const BlockInfo wb = E.blocks[E.k0 + blockIdx.x * blockDim.x + (threadIdx.x & ~63u) + src];
      const uint64_t lo = wb.ustart & ~127ull;
      const uint64_t hi = min(wb.ustart + wb.isize + 4096, E.e_inf);
      for (uint64_t a = lo + 128ull * lane; a < hi; a += 128ull * 64) acc += ldu32(E.u, a);
    }
    if (acc == 0x9e3779b9u && E.k0 == 0xffffffffu) atomicOr(overflow, 0u);  // keeps the loads (never true)
  }
  if (i >= nb) return;
  uint64_t f = kNone;  // guess
  if (force) {
    f = force[i];
    if (f == kNone) return;  // keep this block's walk
  }
  const BlockInfo b = E.blocks[E.k0 + i];
  const uint64_t bend = b.ustart + b.isize;
  if (validate && f != kForceEmpty && f != kNone) {
    // a link-round entry may itself come from a wrong walk upstream (fixed in
    // the same round): re-walk only if the chain from it is plausible to the
    // block end and beyond; otherwise keep the old walk for the next round
    uint64_t q = f;
    bool ok = true;
    int extra = 0;
    while (ok) {
      if (q >= bend && (extra++ >= kGuessLookahead || q == E.e_true || q + 36 > E.e_inf)) break;
      if (!plausible(E, q)) ok = false;
      else q += 4 + (uint64_t)(int32_t)ldu32(E.u, q);
    }
    if (!ok) return;
  }
  uint16_t* __restrict__ L = list + (uint64_t)i * kListCap;
  uint64_t g = kNone, x = kNone;
  uint32_t n = 0;
  bool plaus_list = false;  // every listed record passed plausible()
  const bool live = bend > E.p0 && b.ustart < E.q_end && b.isize > 0;
  if (live && f != kForceEmpty) {
    uint64_t entry = f;
    if (f == kNone && b.ustart <= E.p0) entry = E.p0;  // the block of the span start: entry known
    if (entry != kNone) {
      g = entry;
      uint64_t q = entry, nq;
      while (q < bend) {
        if (n < kListCap) L[n] = (uint16_t)(q - b.ustart);
        ++n;
        if (!chain_step<MODE>(E, q, &nq)) break;
        q = nq;
      }
      x = q;
    } else {
      const uint64_t c = cand[i];
      if (c < bend) {  // c == kNone (no candidate): nothing to walk
        // software-pipelined: record q's read-name end byte and the next
        // record's head are loaded together (plausible_head), one dependent
        // round trip per record.  Loads past the inflated range read the
        // stream's padding and are not used (plausible_head's rules).
        uint64_t q = c, exitq = c;
        uint32_t m = 0;
        bool valid = true;
        RecHead h = load_head(E.u, q);
        int left = kGuessLookahead;  // plausible records required past the block end
        for (;;) {
          const bool inside = q < bend;
          if (!inside && (left-- <= 0 || q == E.e_true || q + 36 > E.e_inf)) break;
          uint64_t na = q;
          const int ph = plausible_head(E, q, h, &na);
          const uint64_t q2 = q + 4 + (uint64_t)(int32_t)h.at(0);
          const uint8_t nb = E.u[na];
          // (q2 may lie anywhere: its head is loaded when its block_size is
          // inflated; reads reach 40 bytes past it, inside the stream's pad)
          h = load_head(E.u, q2 + 4 <= E.e_inf ? q2 : q);
          if (ph == 0 || (ph == 2 && nb != 0)) { valid = false; break; }
          if (inside) {
            if (m < kListCap) L[m] = (uint16_t)(q - b.ustart);
            ++m;
            exitq = q2;  // the first record start past the block (the walk's exit)
          }
          q = q2;
        }
        q = exitq;
        if (valid) {
          g = c;
          x = q;
          n = m;
          plaus_list = true;
        } else {
          g = kRetry;  // later candidates: k_rec_search (wave per block)
          n = 0;
        }
      }
    }
  }
  if (n > kListCap) atomicOr(overflow, 1u);
  g_out[i] = g;
  x_out[i] = x;
  wcnt[i] = n | (plaus_list ? kListPlausible : 0u);
}

// Blocks whose first candidate failed (k_rec_walk: g == kRetry): one wave
// per block tries the later candidates in order (64 positions per step, a
// wave-uniform walk per candidate), as BAMSplitGuesser tries candidate after
// candidate; the valid one's records are listed by lane 0.
template <int MODE>
__global__ __launch_bounds__(64) void k_rec_search(ChainEnv E, const uint64_t* __restrict__ cand,
                                                   uint64_t* __restrict__ g_out, uint64_t* __restrict__ x_out,
                                                   uint32_t* __restrict__ wcnt, uint16_t* __restrict__ list,
                                                   uint32_t* __restrict__ overflow) {
  const uint32_t i = blockIdx.x;
  if (g_out[i] != kRetry) return;
  const uint32_t lane = lane_id();
  const BlockInfo b = E.blocks[E.k0 + i];
  const uint64_t bend = b.ustart + b.isize;
  {  // the walks below are dependent-load chains: pull the block (+ the
     // lookahead past its end) into L2 first with independent loads
    uint32_t acc = 0;
    const uint64_t hi = min(bend + 4096, E.e_inf);
    for (uint64_t a = (b.ustart & ~127ull) + 128ull * lane; a < hi; a += 128ull * 64) acc += ldu32(E.u, a);
    if (acc == 0x9e3779b9u && E.k0 == 0xffffffffu) atomicOr(overflow, 0u);  // keeps the loads (never true)
  }
  uint64_t g = kNone, x = kNone;
  for (uint64_t c0 = cand[i] + 1; c0 < bend && g == kNone; c0 += 64) {
    const uint64_t p = c0 + lane;
    const bool pre = p < bend && cand_prefilter(E, p);
    uint64_t m = __ballot(pre) ? __ballot(pre && plausible2(E, p)) : 0ull;
    while (m) {
      const uint64_t c = c0 + (uint64_t)(__ffsll((long long)m) - 1);
      m &= m - 1;
      uint64_t q = c;
      bool valid = true;
      while (q < bend) {
        if (!plausible(E, q)) { valid = false; break; }
        q += 4 + (uint64_t)(int32_t)ldu32(E.u, q);
      }
      if (valid) {
        uint64_t y = q;
        for (int k = 0; k < kGuessLookahead; ++k) {
          if (y == E.e_true || y + 36 > E.e_inf) break;
          if (!plausible(E, y)) { valid = false; break; }
          y += 4 + (uint64_t)(int32_t)ldu32(E.u, y);
        }
      }
      if (valid) {
        g = c;
        x = q;
        break;
      }
    }
  }
  if (lane == 0) {
    uint32_t n = 0;
    if (g != kNone) {
      uint16_t* __restrict__ L = list + (uint64_t)i * kListCap;
      for (uint64_t q = g; q < bend; q += 4 + (uint64_t)(int32_t)ldu32(E.u, q)) {
        if (n < kListCap) L[n] = (uint16_t)(q - b.ustart);
        ++n;
      }
      if (n > kListCap) atomicOr(overflow, 1u);
    }
    g_out[i] = g;
    x_out[i] = x;
    wcnt[i] = n | (g != kNone ? kListPlausible : 0u);
  }
}

// Parallel link check (in = exclusive max-scan of the guess exits).  Entries
// where the chain enters a block; a block whose walk does not start there is
// re-walked from it (force = entry), a stray walk in a pass-through block is
// dropped (force = kForceEmpty).  A chain that breaks before a block is a
// hard violation (serial link).
__global__ void k_rec_linkfix(ChainEnv E, const uint64_t* __restrict__ g, const uint64_t* __restrict__ x,
                              const uint64_t* __restrict__ in_scan, uint64_t* __restrict__ entry,
                              uint64_t* __restrict__ force, uint32_t* __restrict__ counters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nb = E.k1 - E.k0;
  if (i >= nb) return;
  if (i == 0) {
    entry[0] = E.p0;
    const BlockInfo b = E.blocks[E.k0];
    if (x[0] < b.ustart + b.isize) atomicAdd(&counters[0], 1u);  // chain stops in the first block
    return;
  }
  const BlockInfo b = E.blocks[E.k0 + i];
  const uint64_t bend = b.ustart + b.isize;
  const uint64_t in = in_scan[i];
  const uint64_t gi = g[i];
  uint64_t e = kNone;
  if (in >= E.q_end) {
    e = kNone;
  } else if (in >= bend || b.isize == 0) {
    if (gi != kNone && x[i] > in) {  // a stray walk would corrupt later in[]
      force[i] = kForceEmpty;
      atomicAdd(&counters[1], 1u);
    }
  } else if (in < b.ustart) {
    atomicAdd(&counters[0], 1u);  // a block before stopped inside itself
  } else {
    e = in;
    if (gi != in) {
      force[i] = in;
      atomicAdd(&counters[1], 1u);
    }
  }
  entry[i] = e;
}

// force[] off the serial link's entry[]
__global__ void k_force_from_entry(const uint64_t* __restrict__ g, const uint64_t* __restrict__ entry, uint32_t nb,
                                   uint64_t* __restrict__ force) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const uint64_t e = entry[i], gi = g[i];
  force[i] = e == gi ? kNone : (e == kNone ? kForceEmpty : e);
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// The k_rec_count rules for the listed record at q (one lane): *stop = the
// block's count ends at this record (*counted: the record itself counts),
// *s = its status, *nd = bytes past the inflated range the record needs,
// *long_cigar = its cigar was left to record_invalid_wave.
template <int MODE>
__device__ __forceinline__ void check_listed_h(const ChainEnv& E, uint64_t q, uint64_t lim, bool first, bool light,
                                               bool* stop, bool* counted, int* s, uint64_t* nd, bool* long_cigar,
                                               const RecHead& h) {
  const uint64_t avail = E.e_true - q;
  if (q >= lim) {
    *stop = true;  // outside the span
  } else if (light && !dead_near(E, q)) {
    // all rules pass without reading the record
  } else if (MODE == kReader) {
    if (!first && is_dead(E, q)) {
      *stop = true;  // readInt at an exhausted block + empty block: EOF
    } else if (avail < 4) {
      *stop = true;
    } else if (q + 4 > E.e_inf) {
      *stop = true;
      *nd = q + 4;
    } else {
      const int32_t bs = (int32_t)h.at(0);
      if (bs < 32) {
        *stop = true;
        *s = kErrFormat;
      } else if (dead_in_record(E, q, bs) || avail - 4 < (uint64_t)bs) {
        *stop = true;
        *s = kErrTrunc;
      } else if (q + 4 + (uint64_t)bs > E.e_inf) {
        *stop = true;
        *nd = q + 4 + (uint64_t)bs;
      } else {
        const int32_t ref = (int32_t)h.at(1), nref = (int32_t)h.at(6);
        if (ref < -1 || ref >= E.n_ref || nref < -1 || nref >= E.n_ref) {
          *stop = true;
          *s = kErrArg;
        } else if (E.validate && record_invalid_h(E, q, bs, E.validate == 2, long_cigar, h)) {
          *stop = true;
          *s = kErrFormat;
        }
      }
    }
  } else {
    if (is_dead(E, q)) {
      *stop = true;
    } else if (avail < 4) {
      *stop = true;
      if (avail > 0) *s = kErrIO;  // "less than 4 bytes long"
    } else if (q + 4 > E.e_inf) {
      *stop = true;
      *nd = q + 4;
    } else {
      const int32_t bs = (int32_t)h.at(0);
      if (bs > 0 && ((uint64_t)bs > avail - 4 || is_dead(E, q + 4))) {
        *stop = true;
        *counted = true;
        *s = kErrIO;  // "Skip failed"
      }
    }
  }
}
// Record check and output in one pass (the list path of decode_span_pos):
// the record rules, the long-cigar validation and the output, one wave per
// block, so a block's records are read from HBM once after inflate and
// written out while they are in L2.  A block writes its records at base[i],
// the exclusive scan of the lists' counts: the true offsets for every block
// up to the first one that stops early, since every block before it keeps
// its whole list.  A stop ends the reader's iteration (a failure, EOF at an
// empty block, the end of the stream or of the span) and the indexer's, so
// the span's records are exactly those up to the first stop, and what later
// blocks write lies past them.  The launch reports:
//   bad[0]   min over blocks that stop early or fail of (i << 40 | base[i] +
//            count): the first such block and the records up to its stop
//   flags[0] the first failing block (its status is the span's when it is
//            the first stop)
//   cnt[] / err[] per block, need = the bytes a stopped record needs past
//            the inflated range.
constexpr int kBadShift = 40;

// (4 / 6 / 8 waves per SIMD: 1.116 / 1.065 / 1.052 ms per C2 pass,
// profiles/r06_late/variants_check_out_waves.log)
template <int MODE, bool DECODE>
__global__ __launch_bounds__(64, 6) void k_rec_check_out(ChainEnv E, const uint64_t* __restrict__ entry,
                                                         const uint32_t* __restrict__ wcnt,
                                                         const uint16_t* __restrict__ list,
                                                         const uint64_t* __restrict__ base, uint32_t* __restrict__ cnt,
                                                         int32_t* __restrict__ err,
                                                         unsigned long long* __restrict__ need,
                                                         unsigned long long* __restrict__ bad,
                                                         uint32_t* __restrict__ flags, uint64_t* __restrict__ rec_pos,
                                                         uint64_t* __restrict__ rec_voff, Columns col, uint64_t cap) {
  const uint32_t lane = lane_id();
  const uint32_t i = blockIdx.x;
  const uint64_t e = entry[i];
  const BlockInfo b = E.blocks[E.k0 + i];
  const uint16_t* __restrict__ L = list + (uint64_t)i * kListCap;
  const uint64_t lim = min(b.ustart + b.isize, E.q_end);
  const uint32_t wc = wcnt[i];
  const uint32_t listed = e == kNone ? 0u : min(wc & kListCountMask, kListCap);
  // (check_block's rules) a plausible() list on fully inflated data already
  // satisfies every rule that reads the record
  const bool light = (wc & kListPlausible) && E.e_inf == E.e_true && (MODE != kReader || E.validate == 0);
  const uint64_t o0 = base[i];
  uint32_t count = listed;
  int st = kOk;
  uint64_t nd = 0;
  // 64 records at a time: check them, validate their long cigars, and write
  // the ones before the first stop while their lines are still in L1/L2 (a
  // whole block checked before any output re-fetched every line: 5.9 GB per
  // C2 pass)
  for (uint32_t r0 = 0; r0 < listed; r0 += 64) {
    const uint32_t r = r0 + lane;
    const uint64_t q = r < listed ? b.ustart + L[r] : 0;
    bool stop = false, counted = false, long_cigar = false;
    int s = kOk;
    uint64_t x = 0;
    // the record's head is loaded once for the checks and the output (three
    // passes over it re-fetched its lines from HBM: 5.3 GB per C2 pass)
    RecHead h{};
    if (r < listed) {
      h = load_head(E.u, q);
      check_listed_h<MODE>(E, q, lim, r == 0 && q == E.p0, light, &stop, &counted, &s, &x, &long_cigar, h);
    }
    uint32_t m = min(64u, listed - r0);  // records of this chunk that stand
    const uint64_t sm = __ballot(stop);
    bool halt = sm != 0;  // the block's count ends in this chunk
    if (sm) {
      const uint32_t f = (uint32_t)__ffsll((long long)sm) - 1;
      m = f + (uint32_t)__shfl((int)counted, (int)f, 64);
      st = __shfl(s, (int)f, 64);
      nd = shfl_u64(x, f);
    }
    if (MODE == kReader) {
      // cigars longer than kWaveCigarOps before the stop, a wave each in order
      // (k_rec_check_long): the first invalid one becomes the stop
      const bool lg = lane < m && long_cigar;
      for (uint64_t wm = __ballot(lg); wm; wm &= wm - 1) {
        const uint32_t src = (uint32_t)__ffsll((long long)wm) - 1;
        const uint64_t qq = shfl_u64(q, src);
        if (record_invalid_wave(E, qq, (int32_t)ldu32(E.u, qq), E.validate == 2)) {
          m = src;
          st = kErrFormat;
          nd = 0;
          halt = true;
          break;
        }
      }
    }
    if (lane < m) {
      const uint64_t o = o0 + r;
      if (o < cap) {  // (sized from the lists' counts: always)
        rec_pos[o] = q;
        rec_voff[o] = (b.coff << 16) | (q - b.ustart);
        if (DECODE) decode_record_h(E.u, q, o, col, h);
      }
    }
    if (halt) {
      count = r0 + m;
      break;
    }
  }
  if (lane == 0) {
    if (nd) atomicMax(need, (unsigned long long)nd);
    cnt[i] = count;
    err[i] = st;
    if (count < listed || st != kOk)
      atomicMin(bad, ((unsigned long long)i << kBadShift) | (unsigned long long)(o0 + count));
    if (st != kOk) atomicMin(&flags[0], i);
    // (no per-block atomic on a shared word here: 52 K of them on one address
    // serialize across the XCDs; k_records_after answers for the rare stop)
  }
}

// *flag = 1 when a block after block k has records (a span cut at an early
// stop dropped them: a diagnostic, hbam_pipeline_counters)
__global__ void k_records_after(const uint32_t* __restrict__ cnt, uint32_t nb, uint32_t k, uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > k && i < nb && cnt[i]) *flag = 1u;
}
hipError_t launch_records_after(const uint32_t* cnt, uint32_t nb, uint32_t k, uint32_t* flag, hipStream_t s) {
  hipLaunchKernelGGL(k_records_after, dim3((nb + 255) / 256), dim3(256), 0, s, cnt, nb, k, flag);
  return hipGetLastError();
}

// first block (index) whose status is non-zero -> *first (atomicMin), status -> code[]
__global__ void k_first_error_hout(const HuffOut* __restrict__ hout, uint32_t b0, uint32_t nb,
                                   uint32_t* __restrict__ first) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && hout[b0 + i].status != kOk) atomicMin(first, i);
}
__global__ void k_first_error_i32(const int32_t* __restrict__ err, uint32_t nb, uint32_t* __restrict__ first) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && err[i] != kOk) atomicMin(first, i);
}
// zero the counts of blocks after `cut` (the first failing block)
__global__ void k_truncate_counts(uint32_t* __restrict__ cnt, uint32_t nb, const uint32_t* __restrict__ cut) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && i > *cut) cnt[i] = 0;
}

// .splitting-bai (SplittingBAMIndexer.java:273-277): the voff of every record
// whose global ordinal go = o0 + o satisfies (go + 1) % g == 0, at index
// (go + 1) / g - 1 - o0 / g (entries of earlier windows come before).
__global__ void k_sbi_emit(const uint64_t* __restrict__ voff, uint64_t n, uint32_t g, uint64_t o0,
                           uint64_t* __restrict__ ent) {
  const uint64_t k0 = o0 / g;
  for (uint64_t o = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; o < n;
       o += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t go = o0 + o;
    if ((go + 1) % g == 0) ent[(go + 1) / g - 1 - k0] = voff[o];
  }
}

// the chain successor of the last record of a span: where the next window
// (or the next batch of a split) resumes
__global__ void k_next_pos(const uint8_t* __restrict__ u, const uint64_t* __restrict__ rec_pos, uint64_t n,
                           uint64_t p0, int mode, uint64_t* __restrict__ out, SpecGate gate) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (gate_closed(gate)) return;
  if (n == 0) {
    *out = p0;
    return;
  }
  const uint64_t q = rec_pos[n - 1];
  const int32_t bs = (int32_t)ldu32(u, q);
  *out = q + 4 + (uint64_t)(mode == kReader ? bs : (bs > 0 ? bs : 0));
}

// Digests of a span (bench / test parity checks, not on the timed path):
// out[0] xor of the keys, out[1] sum of the voffs (order-independent), and
// the order-sensitive out[2] / out[3] = sum_i dmix(x_i) * P^(n-1-i) mod 2^64
// over keys / voffs (oracle/hbam_oracle.h ORC_DIGEST_P; composable across
// windows and ranks: D(A ++ B) = D(A) * P^|B| + D(B)).  Each thread takes a
// contiguous run of records (Horner), weighted by P^(records after the run).
__device__ __forceinline__ uint64_t dig_mix(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ uint64_t dig_pow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  for (; e; e >>= 1, b *= b)
    if (e & 1) r *= b;
  return r;
}
constexpr uint64_t kDigestP = 0x100000001b3ull;

__global__ __launch_bounds__(256) void k_digest(const int64_t* __restrict__ keys, const uint64_t* __restrict__ voffs,
                                                uint64_t n, unsigned long long* __restrict__ out) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x, t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t per = (n + nt - 1) / nt;
  const uint64_t i0 = t * per < n ? t * per : n, i1 = i0 + per < n ? i0 + per : n;
  uint64_t kx = 0, vs = 0, kd = 0, vd = 0;
  for (uint64_t i = i0; i < i1; ++i) {
    const uint64_t v = voffs[i];
    vs += v;
    vd = vd * kDigestP + dig_mix(v);
    if (keys) {
      const uint64_t k = (uint64_t)keys[i];
      kx ^= k;
      kd = kd * kDigestP + dig_mix(k);
    }
  }
  const uint64_t w = dig_pow(kDigestP, n - i1);
  kd *= w;
  vd *= w;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    kx ^= (uint64_t)__shfl_xor((unsigned long long)kx, d, 64);
    vs += (uint64_t)__shfl_xor((unsigned long long)vs, d, 64);
    kd += (uint64_t)__shfl_xor((unsigned long long)kd, d, 64);
    vd += (uint64_t)__shfl_xor((unsigned long long)vd, d, 64);
  }
  if (lane_id() == 0) {
    atomicXor(&out[0], (unsigned long long)kx);
    atomicAdd(&out[1], (unsigned long long)vs);
    atomicAdd(&out[2], (unsigned long long)kd);
    atomicAdd(&out[3], (unsigned long long)vd);
  }
}

// ---------------------------------------------------------------------------
// Drop-in batch path (hbam_decode_span): a decoded window's records leave the
// pipeline's buffers for an export slot (so the next window decodes while
// this one's batches cross PCIe; the batches go to the host by SDMA copies
// of column slices).  HBM-bound copy, one thread per record: every column's
// stores coalesce across the wave.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void copy_record_fields(const Columns& s, uint64_t i, const Columns& d, uint64_t j,
                                                   uint64_t rest_base) {
  d.key[j] = s.key[i];
  d.rest_off[j] = s.rest_off[i] - rest_base;
  d.voff[j] = s.voff[i];
  d.ref_id[j] = s.ref_id[i];
  d.pos[j] = s.pos[i];
  d.l_seq[j] = s.l_seq[i];
  d.next_ref_id[j] = s.next_ref_id[i];
  d.next_pos[j] = s.next_pos[i];
  d.tlen[j] = s.tlen[i];
  d.rest_len[j] = s.rest_len[i];
  d.bin[j] = s.bin[i];
  d.n_cigar[j] = s.n_cigar[i];
  d.flag[j] = s.flag[i];
  d.l_read_name[j] = s.l_read_name[i];
  d.mapq[j] = s.mapq[i];
}

// Device -> page-locked host bytes written by the shader engines: a host
// read-back that never waits behind copy-engine traffic of other streams (a
// pageable hipMemcpy D2H of the block table queued ~13 ms behind a drop-in
// batch's D2H on another stream).
__global__ __launch_bounds__(256) void k_readback(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                  uint64_t n) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const uint64_t n16 = n >> 4;
    for (uint64_t i = t; i < n16; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (uint64_t i = (n16 << 4) + t; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < n; i += stride) dst[i] = src[i];
  }
}

// host[i] <- *src[i] for i < n (n <= kGatherMax): a few scattered values read
// back by one launch, with no DMA-engine copy to queue behind larger ones
struct U64Srcs {
  const uint64_t* p[kGatherMax];
};
__global__ __launch_bounds__(64) void k_gather_u64(uint64_t* __restrict__ dst, U64Srcs src, int n) {
  const int i = threadIdx.x;
  if (i < n) dst[i] = *src.p[i];
}

// slot <- records [0, n) of a span; positions rebased so that window position
// `base` (the first record's start) is slot byte 0; dpos[n] = the slot's bytes
// Also (packed != nullptr) the columns once more, batch-major: the records
// [b*m, b*m + m) of batch b as one ColLayout(m) block at packed + b * lf.bytes
// (the last, shorter batch as ColLayout(n - b*m) = ll), with rest_off counted
// in the packed rests (k_pack_rests) from the batch's first record -- exactly
// a drop-in host slot's column area, so a batch's columns cross PCIe as one
// copy instead of fifteen.
__global__ __launch_bounds__(256) void k_export_records(Columns s, const uint64_t* __restrict__ spos, Columns d,
                                                        uint64_t* __restrict__ dpos, uint64_t n, uint64_t base,
                                                        uint64_t nbytes, uint8_t* __restrict__ packed, ColLayout lf,
                                                        ColLayout ll, uint64_t m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    copy_record_fields(s, i, d, i, base);
    dpos[i] = spos[i] - base;
    if (packed) {
      const uint64_t b = i / m, j = i - b * m;
      const bool last = (b + 1) * m > n;
      const Columns c = (last ? ll : lf).at(packed + b * lf.bytes, nullptr);
      copy_record_fields(s, i, c, j, spos[b * m]);
      c.rest_off[j] -= 36 * (j + 1);  // into the batch's packed rests (k_pack_rests)
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) dpos[n] = nbytes;
}

// ---------------------------------------------------------------------------
// SAMRecordWritable codec (SAMRecordWritable.java:55-68)
// ---------------------------------------------------------------------------
// write(): [htsjdk] BAMRecordCodec.encode of an unmodified BAMRecord emits
// block_size (= 32 + rest length), the fixed fields and the undecoded rest --
// the record's own bytes, except that indexBin is written as 0 when refID < 0.
// The records of a span lie back to back in the inflated stream, so the
// encodings of a span are u[p0, p0+n) copied into a 16 B-aligned buffer
// (k_wr_copy: HBM-bound, 2 B of traffic per byte) followed by the sparse bin
// patches (k_wr_bin_patch: 6 B of columns per record).

// 16 bytes starting sh bytes into the 32-byte pair (a, b); sh is uniform.
__device__ __forceinline__ uint4 shift16(const uint4 a, const uint4 b, uint32_t sh) {
  const uint32_t r = sh & 3;
  uint32_t w0, w1, w2, w3, w4;
  switch (sh >> 2) {
    case 0: w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; break;
    case 1: w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; break;
    case 2: w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; break;
    default: w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                    __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r));
}

// Drop-in batches carry each record's rest only (read name .. aux): the 36
// bytes of block_size + fixed fields are in the columns already, and leaving
// them out cuts a batch's D2H by ~10 % (the drop-in loop is PCIe-bound).
// dst <- the rests of records [0, n) of a span, back to back: record i's rest
// lands at cp(i) = rest_off[i] - p0 - 36 (i + 1) (records are contiguous from
// p0, so cp(i + 1) = cp(i) + rest_len[i]).  A workgroup takes 256 records:
// their cp() in LDS, then 16-byte output chunks, each a shifted 16 B load
// when the chunk lies in one rest (most of them) and bytes otherwise.
constexpr uint32_t kPackRecs = 256;
__global__ __launch_bounds__(256) void k_pack_rests(const uint8_t* __restrict__ u,
                                                    const uint64_t* __restrict__ rest_off,
                                                    const uint32_t* __restrict__ rest_len, uint64_t n, uint64_t p0,
                                                    uint8_t* __restrict__ dst) {
  __shared__ uint64_t cp[kPackRecs + 1];
  const uint64_t r0 = (uint64_t)blockIdx.x * kPackRecs;
  if (r0 >= n) return;
  const uint32_t cnt = (uint32_t)min<uint64_t>(kPackRecs, n - r0), t = threadIdx.x;
  if (t < cnt) {
    const uint64_t c = rest_off[r0 + t] - p0 - 36 * (r0 + t + 1);
    cp[t] = c;
    if (t == cnt - 1) cp[cnt] = c + rest_len[r0 + t];
  }
  __syncthreads();
  const uint64_t lo = cp[0], hi = cp[cnt];
  const uint64_t skew = p0 + 36 * (r0 + 1);  // source = output + skew + 36 * (local record)
  for (uint64_t c = (lo & ~15ull) + 16ull * t; c < hi; c += 16ull * blockDim.x) {
    const uint64_t o0 = max(c, lo), o1 = min(c + 16, hi);
    uint32_t a = 0, b = cnt - 1;  // the last record with cp <= o0
    while (a < b) {
      const uint32_t mid = (a + b + 1) >> 1;
      if (cp[mid] <= o0) a = mid; else b = mid - 1;
    }
    if (o0 == c && o1 == c + 16 && cp[a + 1] >= c + 16) {
      const uint64_t src = c + skew + 36ull * a;
      const uint4* q = reinterpret_cast<const uint4*>(u + (src & ~15ull));
      *reinterpret_cast<uint4*>(dst + c) = shift16(q[0], q[1], (uint32_t)(src & 15));
    } else {
      for (uint64_t o = o0; o < o1; ++o) {
        while (cp[a + 1] <= o) ++a;
        dst[o] = u[o + skew + 36ull * a];
      }
    }
  }
}

constexpr int kWrUnroll = 4;  // 16 B chunks in flight per thread
// dst[0, 16*ceil(n/16)) = u[p0, ...): chunk c of the destination comes from
// the aligned source chunks c and c+1 (the stream is padded past its end).
__global__ __launch_bounds__(256) void k_wr_copy(const uint8_t* __restrict__ u, uint64_t p0, uint64_t n,
                                                 uint8_t* __restrict__ dst) {
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(u + (p0 & ~15ull));
  uint4* __restrict__ d = reinterpret_cast<uint4*>(dst);
  const uint32_t sh = (uint32_t)(p0 & 15);
  const uint64_t nch = (n + 15) >> 4;
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; c + (kWrUnroll - 1) * T < nch; c += kWrUnroll * T) {  // kWrUnroll coalesced chunks per thread
    uint4 a[kWrUnroll], b[kWrUnroll];
#pragma unroll
    for (int k = 0; k < kWrUnroll; ++k) {
      a[k] = src[c + k * T];
      b[k] = src[c + k * T + 1];
    }
#pragma unroll
    for (int k = 0; k < kWrUnroll; ++k) d[c + k * T] = shift16(a[k], b[k], sh);
  }
  for (; c < nch; c += T) d[c] = shift16(src[c], src[c + 1], sh);
}

__global__ void k_wr_bin_patch(const uint64_t* __restrict__ rec_pos, const int32_t* __restrict__ ref_id,
                               const uint16_t* __restrict__ bin, uint64_t n, uint64_t p0, uint8_t* __restrict__ dst) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (ref_id[i] < 0 && bin[i] != 0) {  // [htsjdk] encode: indexBin = 0 unless refIndex >= 0
      const uint64_t q = rec_pos[i] - p0 + 14;
      dst[q] = 0;
      dst[q + 1] = 0;
    }
  }
}

// readFields(): [htsjdk] BAMRecordCodec.decode (LazyBAMRecordFactory, no
// header) once per framed value buf[offs[i], offs[i+1]) (the last ends at
// len).  The first failing value's index and status go to *bad
// ((i << 8) | status, atomicMin); values decode independently.
__global__ void k_wr_decode(const uint8_t* __restrict__ buf, uint64_t len, const uint64_t* __restrict__ offs,
                            uint64_t n, Columns col, uint64_t* __restrict__ rec_pos,
                            unsigned long long* __restrict__ bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p = offs[i], e = i + 1 < n ? offs[i + 1] : len;
    uint32_t code = kOk;
    if (e < p || e > len) {
      code = kErrArg;
    } else if (e - p < 4) {
      code = kErrTrunc;  // readInt at EOF: decode() returns null
    } else {
      const int32_t bs = (int32_t)ldu32(buf, p);
      if (bs < 32) code = kErrFormat;                         // "Invalid record length"
      else if (e - p - 4 < (uint64_t)bs) code = kErrTrunc;    // readFully short: RuntimeEOFException
    }
    if (code != kOk) {
      atomicMin(bad, (unsigned long long)((i << 8) | code));
      continue;
    }
    decode_record(buf, p, i, col);
    col.voff[i] = kNone;  // a shuffled record has no file position
    rec_pos[i] = p;
  }
}

// ---------------------------------------------------------------------------
// host launch wrappers (hbam_launch.h)
// ---------------------------------------------------------------------------
static inline unsigned grid_for(uint64_t n, unsigned bs, unsigned cap = 65535u * 4) {
  uint64_t g = (n + bs - 1) / bs;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

hipError_t launch_bgzf_scan(const uint8_t* file, uint64_t buf_base, uint64_t lo, uint64_t hi, uint64_t* cand,
                            uint32_t cap, uint32_t* count, hipStream_t s) {
  // scan from the 16 B aligned file offset at or below lo (windows are placed
  // so that file offsets keep their alignment; the bytes below buf_base are
  // allocated); candidates below lo are dropped
  (void)buf_base;
  const uint64_t a = lo & ~15ull;
  const uint64_t nc = (hi - a + 15) / 16;  // 16 B per lane and step, 4 steps per iteration
  hipLaunchKernelGGL(k_bgzf_scan, dim3(grid_for((nc + 3) / 4, 256, HBAM_SCAN_GRID)), dim3(256), 0, s, file + a, hi - a, a, lo,
                     cand, cap, count);
  return hipGetLastError();
}
hipError_t launch_bgzf_verify(const uint8_t* file, uint64_t lo, uint64_t hi, const uint64_t* cand, uint32_t n,
                              BlockInfo* blocks, uint32_t* flags, uint32_t partial, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bgzf_verify, dim3((n + 255) / 256), dim3(256), 0, s, file, lo, hi, cand, n, blocks, flags,
                     partial);
  return hipGetLastError();
}
hipError_t launch_bgzf_walk(const uint8_t* file, uint64_t lo, uint64_t hi, BlockInfo* blocks, uint32_t cap,
                            uint32_t* out, uint32_t partial, hipStream_t s) {
  hipLaunchKernelGGL(k_bgzf_walk, dim3(1), dim3(64), 0, s, file, lo, hi, blocks, cap, out, partial);
  return hipGetLastError();
}
hipError_t launch_block_ustart(BlockInfo* blocks, uint32_t n, uint64_t* tmp_isize, uint64_t* tmp_ustart,
                               void* scan_tmp, size_t* scan_bytes, uint64_t base, hipStream_t s) {
  if (scan_tmp == nullptr) {  // size query
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *scan_bytes, tmp_isize, tmp_ustart, (int)n, s);
  }
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_block_isize, dim3((n + 255) / 256), dim3(256), 0, s, blocks, n, tmp_isize);
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, *scan_bytes, tmp_isize, tmp_ustart, (int)n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_block_ustart, dim3((n + 255) / 256), dim3(256), 0, s, blocks, n, tmp_ustart, base);
  return hipGetLastError();
}
hipError_t sort_u64(void* tmp, size_t* tmp_bytes, uint64_t* keys_in, uint64_t* keys_out, uint32_t n,
                    hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(tmp, *tmp_bytes, keys_in, keys_out, (int)n, 0, 64, s);
}
hipError_t scan_u32_to_u64(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint64_t* out, uint32_t n,
                           hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, in, out, (int)n, s);
}

hipError_t launch_huff_tables(const uint8_t* file, const BlockInfo* blocks, uint32_t b0, uint32_t nb,
                              uint8_t* tables, HuffTableInfo* tinfo, const HuffOut* hout, uint32_t round,
                              hipStream_t s) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_huff_tables, dim3(nb), dim3(64), 0, s, file, blocks, b0, tables, tinfo, hout, round);
  return hipGetLastError();
}
// phase A proper; the chunk's tables must be built (launch_huff_tables).
hipError_t launch_inflate_huff_prebuilt(const uint8_t* file, const BlockInfo* blocks, uint32_t b0, uint32_t nb,
                                        uint64_t chunk_ustart, uint32_t* tokens, HuffOut* hout,
                                        const uint8_t* tables, const HuffTableInfo* tinfo, uint32_t round,
                                        uint32_t defer, hipStream_t s) {
  // (every workgroup decides for its own block whether it stages it, k_inflate_huff)
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_inflate_huff, dim3(nb), dim3(kHuffThreads), 0, s, file, blocks, b0, chunk_ustart, tokens,
                     hout, tables, tinfo, round, defer);
  return hipGetLastError();
}
hipError_t launch_inflate_lz77(const BlockInfo* blocks, uint32_t b0, uint32_t nb, uint64_t chunk_ustart,
                               const uint32_t* tokens, const HuffOut* hout, uint8_t* u, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_inflate_lz77, dim3(nb), dim3(kLzThreads), 0, s, blocks, b0, chunk_ustart, tokens, hout, u);
  return hipGetLastError();
}

hipError_t launch_chain(const ChainArgs& a, int mode, int stage, hipStream_t s) {
  ChainEnv E;
  E.u = a.u;
  E.blocks = a.blocks;
  E.e_inf = a.e_inf;
  E.e_true = a.e_true;
  E.p0 = a.p0;
  E.q_end = a.q_end;
  E.dead = a.dead;
  E.ndead = a.ndead;
  E.n_ref = a.n_ref;
  E.k0 = a.k0;
  E.k1 = a.k1;
  E.validate = a.validate;
  E.ref_len = a.ref_len;
  const uint32_t nb = a.k1 - a.k0;
  if (nb == 0) return hipSuccess;
  const unsigned tb = 64, gb = (nb + tb - 1) / tb;
  switch (stage) {
    case kStageSerialLink:
      if (mode == kReader) hipLaunchKernelGGL(k_rec_link<kReader>, dim3(1), dim3(256), 0, s, E, a.g, a.x, a.entry, a.summary);
      else hipLaunchKernelGGL(k_rec_link<kIndexer>, dim3(1), dim3(256), 0, s, E, a.g, a.x, a.entry, a.summary);
      break;
    case kStageCount:
      if (mode == kReader) hipLaunchKernelGGL(k_rec_count<kReader>, dim3(gb), dim3(tb), 0, s, E, a.entry, a.cnt, a.err, a.need);
      else hipLaunchKernelGGL(k_rec_count<kIndexer>, dim3(gb), dim3(tb), 0, s, E, a.entry, a.cnt, a.err, a.need);
      break;
    case kStageEmit:
      if (mode == kReader) hipLaunchKernelGGL(k_rec_emit<kReader>, dim3(gb), dim3(tb), 0, s, E, a.entry, a.cnt, a.base, a.rec_pos, a.rec_voff);
      else hipLaunchKernelGGL(k_rec_emit<kIndexer>, dim3(gb), dim3(tb), 0, s, E, a.entry, a.cnt, a.base, a.rec_pos, a.rec_voff);
      break;
    case kStageWalk: {  // candidates + walks
      if (mode == kReader) {
        hipLaunchKernelGGL(k_rec_cand<kReader>, dim3(nb), dim3(64), 0, s, E, a.cand);
        hipLaunchKernelGGL(k_rec_walk<kReader>, dim3((nb + 255) / 256), dim3(256), 0, s, E, a.cand, nullptr, a.g,
                           a.x, a.wcnt, a.list, a.counters + 2, false);
        hipLaunchKernelGGL(k_rec_search<kReader>, dim3(nb), dim3(64), 0, s, E, a.cand, a.g, a.x, a.wcnt, a.list,
                           a.counters + 2);
      } else {
        hipLaunchKernelGGL(k_rec_cand<kIndexer>, dim3(nb), dim3(64), 0, s, E, a.cand);
        hipLaunchKernelGGL(k_rec_walk<kIndexer>, dim3((nb + 255) / 256), dim3(256), 0, s, E, a.cand, nullptr, a.g,
                           a.x, a.wcnt, a.list, a.counters + 2, false);
        hipLaunchKernelGGL(k_rec_search<kIndexer>, dim3(nb), dim3(64), 0, s, E, a.cand, a.g, a.x, a.wcnt, a.list,
                           a.counters + 2);
      }
      break;
    }
    case kStageLinkCheck: {  // y, exclusive max-scan, check with re-walk requests
      hipError_t e = hipMemsetAsync(a.force, 0xff, (size_t)nb * 8, s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_rec_link_y, dim3(gb), dim3(tb), 0, s, a.g, a.x, nb, a.x2);
      size_t sb = a.scan_bytes;
      e = hipcub::DeviceScan::ExclusiveScan(a.scan_tmp, sb, a.x2, a.base, hipcub::Max(), (uint64_t)0, (int)nb, s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_rec_linkfix, dim3(gb), dim3(tb), 0, s, E, a.g, a.x, a.base, a.entry, a.force, a.counters);
      break;
    }
    case kStageRewalk:       // re-walk the requested blocks (entries validated)
    case kStageRewalkAll: {  // force off the serial link's (exact) entry[], then re-walk
      const bool validate = stage == kStageRewalk;
      if (stage == kStageRewalkAll) hipLaunchKernelGGL(k_force_from_entry, dim3(gb), dim3(tb), 0, s, a.g, a.entry, nb, a.force);
      if (mode == kReader)
        hipLaunchKernelGGL(k_rec_walk<kReader>, dim3((nb + 255) / 256), dim3(256), 0, s, E, a.cand, a.force, a.g,
                           a.x, a.wcnt, a.list, a.counters + 2, validate);
      else
        hipLaunchKernelGGL(k_rec_walk<kIndexer>, dim3((nb + 255) / 256), dim3(256), 0, s, E, a.cand, a.force, a.g,
                           a.x, a.wcnt, a.list, a.counters + 2, validate);
      break;
    }
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// *total += sum over blocks with an entry of their listed records (capped at kListCap)
// cnt[i] = the records block i's list holds (0 off the chain): the
// optimistic output counts k_rec_check_out's offsets are scanned from
__global__ void k_list_counts(const uint64_t* __restrict__ entry, const uint32_t* __restrict__ wcnt, uint32_t nb,
                              uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) cnt[i] = entry[i] != kNone ? min(wcnt[i] & kListCountMask, kListCap) : 0u;
}

static ChainEnv chain_env(const ChainArgs& a) {
  ChainEnv E;
  E.u = a.u;
  E.blocks = a.blocks;
  E.e_inf = a.e_inf;
  E.e_true = a.e_true;
  E.p0 = a.p0;
  E.q_end = a.q_end;
  E.dead = a.dead;
  E.ndead = a.ndead;
  E.n_ref = a.n_ref;
  E.k0 = a.k0;
  E.k1 = a.k1;
  E.validate = a.validate;
  E.ref_len = a.ref_len;
  return E;
}

hipError_t launch_list_counts(const ChainArgs& a, hipStream_t s) {
  const uint32_t nb = a.k1 - a.k0;
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_list_counts, dim3((nb + 255) / 256), dim3(256), 0, s, a.entry, a.wcnt, nb, a.cnt);
  return hipGetLastError();
}

hipError_t launch_rec_check_out(const ChainArgs& a, int mode, bool decode, const Columns& col, uint64_t cap,
                                hipStream_t s) {
  static_assert(kBadShift == kFusedBadShift, "hbam_launch.h kFusedBadShift");
  const ChainEnv E = chain_env(a);
  const uint32_t nb = a.k1 - a.k0;
  if (nb == 0) return hipSuccess;
  unsigned long long* need = a.need;
  unsigned long long* bad = reinterpret_cast<unsigned long long*>(a.fuse_bad);
#define HBAM_CO(M, D)                                                                                            \
  hipLaunchKernelGGL((k_rec_check_out<M, D>), dim3(nb), dim3(64), 0, s, E, a.entry, a.wcnt, a.list, a.base, a.cnt, \
                     a.err, need, bad, a.fuse_flags, a.rec_pos, a.rec_voff, col, cap)
  if (mode == kReader && decode) HBAM_CO(kReader, true);
  else if (mode == kReader) HBAM_CO(kReader, false);
  else HBAM_CO(kIndexer, false);
#undef HBAM_CO
  return hipGetLastError();
}

hipError_t link_scan_bytes(uint32_t nb, size_t* bytes) {
  uint64_t* p = nullptr;
  return hipcub::DeviceScan::ExclusiveScan(nullptr, *bytes, p, p, hipcub::Max(), (uint64_t)0, (int)nb, (hipStream_t)0);
}

hipError_t launch_rec_decode(const uint8_t* u, const uint64_t* rec_pos, uint64_t n, const Columns& col,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rec_decode, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, u, rec_pos, n, col);
  return hipGetLastError();
}
hipError_t launch_first_error_hout(const HuffOut* hout, uint32_t b0, uint32_t nb, uint32_t* first, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_first_error_hout, dim3((nb + 255) / 256), dim3(256), 0, s, hout, b0, nb, first);
  return hipGetLastError();
}
hipError_t launch_first_error_i32(const int32_t* err, uint32_t nb, uint32_t* first, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_first_error_i32, dim3((nb + 255) / 256), dim3(256), 0, s, err, nb, first);
  return hipGetLastError();
}
hipError_t launch_truncate_counts(uint32_t* cnt, uint32_t nb, const uint32_t* cut, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(k_truncate_counts, dim3((nb + 255) / 256), dim3(256), 0, s, cnt, nb, cut);
  return hipGetLastError();
}
hipError_t launch_sbi_emit(const uint64_t* voff, uint64_t n, uint32_t g, uint64_t o0, uint64_t* ent, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sbi_emit, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, voff, n, g, o0, ent);
  return hipGetLastError();
}
hipError_t launch_next_pos(const uint8_t* u, const uint64_t* rec_pos, uint64_t n, uint64_t p0, int mode,
                           uint64_t* out, hipStream_t s, const unsigned long long* gate_bad,
                           const unsigned long long* gate_need, uint64_t gate_e_inf) {
  SpecGate g;
  g.bad = gate_bad;
  g.need = gate_need;
  g.e_inf = gate_e_inf;
  hipLaunchKernelGGL(k_next_pos, dim3(1), dim3(64), 0, s, u, rec_pos, n, p0, mode, out, g);
  return hipGetLastError();
}
hipError_t launch_readback(void* dst, const void* src, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_readback, dim3(grid_for((n + 15) / 16, 256, 64)), dim3(256), 0, s,
                     static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
  return hipGetLastError();
}
hipError_t launch_pack_rests(const uint8_t* u, const uint64_t* rest_off, const uint32_t* rest_len, uint64_t n,
                             uint64_t p0, uint8_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_rests, dim3((unsigned)((n + kPackRecs - 1) / kPackRecs)), dim3(256), 0, s, u, rest_off,
                     rest_len, n, p0, dst);
  return hipGetLastError();
}
hipError_t launch_gather_u64(uint64_t* dst, const uint64_t* const* src, int n, hipStream_t s) {
  if (n <= 0 || n > kGatherMax) return n == 0 ? hipSuccess : hipErrorInvalidValue;
  U64Srcs g{};
  for (int i = 0; i < n; ++i) g.p[i] = src[i];
  hipLaunchKernelGGL(k_gather_u64, dim3(1), dim3(64), 0, s, dst, g, n);
  return hipGetLastError();
}
hipError_t launch_export_records(const Columns& src, const uint64_t* src_pos, const Columns& dst, uint64_t* dst_pos,
                                 uint64_t n, uint64_t base, uint64_t nbytes, uint8_t* packed, uint64_t m,
                                 hipStream_t s) {
  const ColLayout lf(m ? m : 1, false), ll(m ? n - (n ? (n - 1) / m : 0) * m : 1, false);
  hipLaunchKernelGGL(k_export_records, dim3(grid_for(std::max<uint64_t>(n, 1), 256, 8192)), dim3(256), 0, s, src,
                     src_pos, dst, dst_pos, n, base, nbytes, m ? packed : nullptr, lf, ll, m ? m : 1);
  return hipGetLastError();
}
hipError_t launch_digest(const int64_t* keys, const uint64_t* voffs, uint64_t n, uint64_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_digest, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, keys, voffs, n,
                     reinterpret_cast<unsigned long long*>(out));
  return hipGetLastError();
}
hipError_t launch_wr_encode(const uint8_t* u, uint64_t p0, uint64_t nbytes, const uint64_t* rec_pos,
                            const int32_t* ref_id, const uint16_t* bin, uint64_t n, uint8_t* dst, hipStream_t s) {
  if (nbytes) {
    const uint64_t nch = (nbytes + 15) >> 4;
    // 8 workgroups of 256 per CU (2048 lanes x kWrUnroll chunks in flight each)
    const uint64_t grid = std::min<uint64_t>((nch + 255) / 256, 256ull * 8);
    hipLaunchKernelGGL(k_wr_copy, dim3((unsigned)std::max<uint64_t>(grid, 1)), dim3(256), 0, s, u, p0, nbytes, dst);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wr_bin_patch, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, rec_pos, ref_id, bin, n, p0,
                     dst);
  return hipGetLastError();
}
hipError_t launch_long_hash(const uint8_t* u, const uint64_t* rec_pos, const Columns& col, hipStream_t s,
                            const unsigned long long* gate_bad, const unsigned long long* gate_need,
                            uint64_t gate_e_inf) {
  if (!col.long_rec || col.long_cap == 0) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>(col.long_cap, 256u * 16u);
  SpecGate g;
  g.bad = gate_bad;
  g.need = gate_need;
  g.e_inf = gate_e_inf;
  hipLaunchKernelGGL(k_long_hash, dim3(grid), dim3(64), 0, s, u, rec_pos, col, g);
  return hipGetLastError();
}
hipError_t launch_wr_decode(const uint8_t* buf, uint64_t len, const uint64_t* offs, uint64_t n, const Columns& col,
                            uint64_t* rec_pos, unsigned long long* bad, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wr_decode, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, buf, len, offs, n, col, rec_pos,
                     bad);
  return hipGetLastError();
}

}  // namespace hbam
