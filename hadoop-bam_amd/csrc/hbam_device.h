// hbam_device.h -- device data layout shared by the gfx950 kernels and the host pipeline.
//
// Layout in HBM (one pipeline = one GPU):
//   file    : the compressed BGZF bytes, resident, padded with kFilePad zero bytes
//   blocks  : BlockInfo[nblocks] (AoS, 32 B) from bgzf_locate
//   u       : the inflated stream, block k at u + ustart_k (contiguous, padded)
//   tokens  : per-chunk LZ77 token stream (phase A -> phase B of inflate)
//   records : rec_pos / voff / SoA columns (one slot per record of the span)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbam {

constexpr uint64_t kFilePad = 8192;      // zero bytes after the file (ring prefetch)
constexpr uint64_t kUPad = 4096;         // zero bytes after the inflated stream
constexpr uint32_t kMaxIsize = 65536;    // BGZF ISIZE limit handled on device
constexpr uint64_t kNone = ~0ull;

// status codes (== include/hbam.h)
enum : int {
  kOk = 0,
  kErrFormat = 1,  // SAMFormatException
  kErrTrunc = 2,   // FileTruncatedException / RuntimeEOFException
  kErrArg = 3,     // IllegalArgumentException
  kErrIO = 4,      // IOException / RuntimeIOException (DataFormatException)
  kErrDevice = 5,
  kErrState = 6,
  kErrNoMem = 7,
  // (device-side per-block status, never returned) the block's records end
  // the iteration without an error: EOF at an empty block after an exhausted
  // one, or the end of the stream (k_rec_count)
  kStopClean = -1,
};

struct BlockInfo {
  uint64_t coff;    // compressed offset in the file
  uint64_t ustart;  // offset of the block's first inflated byte in u
  uint32_t csize;   // BSIZE + 1
  uint32_t isize;   // ISIZE footer
  uint32_t crc;     // CRC32 footer
  uint32_t flags;   // reserved
};
static_assert(sizeof(BlockInfo) == 32, "BlockInfo is 32 bytes");

// Per-block result of inflate phase A.
struct HuffOut {
  uint32_t ntok;
  int32_t status;       // kOk, an error code, or kHuffPending between rounds
  uint32_t resume_bit;  // kHuffPending: the next DEFLATE block header (bit, relative to the 16 B-aligned cdata base)
  uint32_t outpos;      // kHuffPending: bytes inflated so far
};
// Phase A runs in rounds: a block whose next DEFLATE block needs a header
// stops there (kHuffPending); the next round's k_huff_tables parses that
// header at high occupancy and the decode resumes with the tables prebuilt.
constexpr int32_t kHuffPending = -2;
#ifndef HBAM_INFLATE_ROUNDS
#define HBAM_INFLATE_ROUNDS 2
#endif
// zlib writes <= 4 DEFLATE blocks of 16383 symbols per 64 KiB BGZF block and
// htslib/bgzip data nearly always 2: rounds 3-4 cost ~47 us of near-empty
// launches per chunk, so a third or fourth header is parsed inline in round 1
constexpr uint32_t kInflateRounds = HBAM_INFLATE_ROUNDS;

// Phase-A table prebuild (k_huff_tables -> k_inflate_huff), per block of a chunk.
constexpr uint32_t kHuffTableImage = 8704;  // bytes of the LDS table image
struct HuffTableInfo {
  uint32_t status;     // 0: tables + B0 valid; else decode the block's headers inline
  uint32_t B0;         // bit of the first symbol (relative to the 16 B-aligned cdata base)
  uint32_t final_blk;  // BFINAL of the first DEFLATE block
  uint32_t est_bits;   // expected compressed bits of that block (block_bits_estimate)
};

// Record-chain transition rules.
enum ChainMode : int {
  kReader = 0,  // [htsjdk] BAMRecordCodec.decode (BAMRecordReader path)
  kIndexer = 1, // SplittingBAMIndexer.readAlignment + fullySkip
};

// Decoded SoA columns of one span (device pointers).  Field set of
// LazyBAMRecordFactory.createBAMRecord (LazyBAMRecordFactory.java:37-50).
struct Columns {
  int32_t *ref_id, *pos, *l_seq, *next_ref_id, *next_pos, *tlen;
  uint8_t *l_read_name, *mapq;
  uint16_t *bin, *n_cigar, *flag;
  int64_t *key;
  uint64_t *voff, *rest_off;
  uint32_t *rest_len;
  // Keys whose Murmur input (the rest) is longer than kLongHash bytes are
  // deferred to k_long_hash (one wave per record): decode appends the record
  // index here (nullptr: hash inline).
  uint64_t* long_rec;
  uint32_t* long_n;
  uint32_t long_cap;
};
constexpr uint32_t kLongHash = 2048;

// n records' columns in one buffer (the drop-in batch path: a decoded
// window's records exported out of the pipeline on the device, and the
// page-locked host batches): 16 B-aligned pieces, widest columns first.
// rec_pos (device slots only) has n + 1 entries, the last = the slot's byte
// count.
struct ColLayout {
  enum : int {
    kKey, kRestOff, kVoff, kRecPos, kRefId, kPos, kLSeq, kNextRefId, kNextPos, kTlen, kRestLen, kBin, kNCigar,
    kFlag, kLReadName, kMapq, kCount
  };
  uint64_t off[kCount];
  uint64_t bytes;
  __host__ __device__ static constexpr uint32_t size_of(int c) {
    return c <= kRecPos ? 8 : c <= kRestLen ? 4 : c <= kFlag ? 2 : 1;
  }
  ColLayout() = default;
  __host__ __device__ ColLayout(uint64_t n, bool rec_pos) {
    uint64_t p = 0;
    for (int c = 0; c < kCount; ++c) {
      off[c] = p;
      const uint64_t k = c == kRecPos ? (rec_pos ? n + 1 : 0) : n;
      p += (k * size_of(c) + 15) & ~15ull;
    }
    bytes = p;
  }
  // the Columns (no long-key list) of a buffer laid out this way
  __host__ __device__ Columns at(uint8_t* b, uint64_t** rec_pos) const {
    Columns c{};
    c.key = reinterpret_cast<int64_t*>(b + off[kKey]);
    c.rest_off = reinterpret_cast<uint64_t*>(b + off[kRestOff]);
    c.voff = reinterpret_cast<uint64_t*>(b + off[kVoff]);
    if (rec_pos) *rec_pos = reinterpret_cast<uint64_t*>(b + off[kRecPos]);
    c.ref_id = reinterpret_cast<int32_t*>(b + off[kRefId]);
    c.pos = reinterpret_cast<int32_t*>(b + off[kPos]);
    c.l_seq = reinterpret_cast<int32_t*>(b + off[kLSeq]);
    c.next_ref_id = reinterpret_cast<int32_t*>(b + off[kNextRefId]);
    c.next_pos = reinterpret_cast<int32_t*>(b + off[kNextPos]);
    c.tlen = reinterpret_cast<int32_t*>(b + off[kTlen]);
    c.rest_len = reinterpret_cast<uint32_t*>(b + off[kRestLen]);
    c.bin = reinterpret_cast<uint16_t*>(b + off[kBin]);
    c.n_cigar = reinterpret_cast<uint16_t*>(b + off[kNCigar]);
    c.flag = reinterpret_cast<uint16_t*>(b + off[kFlag]);
    c.l_read_name = b + off[kLReadName];
    c.mapq = b + off[kMapq];
    return c;
  }
};

}  // namespace hbam
