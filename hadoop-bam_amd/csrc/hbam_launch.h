// hbam_launch.h -- host-callable launch wrappers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbam_device.h"

namespace hbam {

struct ChainArgs {
  const uint8_t* u;
  const BlockInfo* blocks;
  uint64_t e_inf, e_true, p0, q_end;
  const uint64_t* dead;
  uint32_t ndead;
  int32_t n_ref;
  uint32_t k0, k1;
  int validate;            // reader mode: 0 SILENT, 1 LENIENT (decode structure only), 2 STRICT (SAMRecord.isValid)
  const int32_t* ref_len;  // n_ref reference lengths (nullptr: alignment-start bound not checked)
  // per-block scratch (indexed by k - k0)
  uint64_t *g, *x, *entry, *summary, *base;
  uint64_t* x2;        // parallel link: y (walk exits)
  void* scan_tmp;      // parallel link: hipcub temp storage
  size_t scan_bytes;
  uint32_t* cnt;
  int32_t* err;
  unsigned long long* need;
  // outputs
  uint64_t *rec_pos, *rec_voff;
  // lane-per-block walks + per-block record lists
  uint64_t* cand;       // first plausible record start per block
  uint64_t* force;      // re-walk requests (kNone = keep)
  uint32_t* wcnt;       // records listed per block
  uint16_t* list;       // kListCap u16 offsets (from ustart) per block
  uint32_t* counters;   // [0] hard link violations, [1] blocks to re-walk, [2] list overflow
  // fused check + output (launch_rec_check_out)
  uint64_t* fuse_bad;    // = ~0: min (i << kFusedBadShift | records up to i's stop) over blocks that stop early
  uint32_t* fuse_flags;  // [0] first failing block = ~0
};
constexpr uint32_t kListCap = 2048;              // >= 65536 / 36 + 2: every reader-mode record start
constexpr uint64_t kForceEmpty = ~0ull - 1;      // force[]: the block holds no record start

// launch_chain stages
enum ChainStage : int {
  kStageSerialLink = 1,  // exact serial link over the walk exits (entry[] + summary)
  kStageCount = 2,       // per-block count + validation by walking (list overflow path)
  kStageEmit = 3,        // per-block positions + voffs by walking (list overflow path)
  kStageWalk = 5,        // candidates + lane-per-block walks
  kStageLinkCheck = 6,   // max-scan link check with re-walk requests
  kStageRewalk = 7,      // re-walk the requested blocks (entries validated)
  kStageRewalkAll = 8,   // re-walk every block off the serial link's entry[]
};

// candidates in [lo, hi); file + buf_base is the (aligned) device buffer start
hipError_t launch_bgzf_scan(const uint8_t* file, uint64_t buf_base, uint64_t lo, uint64_t hi, uint64_t* cand,
                            uint32_t cap, uint32_t* count, hipStream_t s);
// partial != 0: bytes past hi are not part of the window; a block cut by hi
// ends the range (verify: flags[2] = 1; walk: out[2..3] = its start, status OK)
hipError_t launch_bgzf_verify(const uint8_t* file, uint64_t lo, uint64_t hi, const uint64_t* cand, uint32_t n,
                              BlockInfo* blocks, uint32_t* flags, uint32_t partial, hipStream_t s);
hipError_t launch_bgzf_walk(const uint8_t* file, uint64_t lo, uint64_t hi, BlockInfo* blocks, uint32_t cap,
                            uint32_t* out, uint32_t partial, hipStream_t s);
// ustart = base + exclusive scan of ISIZE
hipError_t launch_block_ustart(BlockInfo* blocks, uint32_t n, uint64_t* tmp_isize, uint64_t* tmp_ustart,
                               void* scan_tmp, size_t* scan_bytes, uint64_t base, hipStream_t s);
hipError_t sort_u64(void* tmp, size_t* tmp_bytes, uint64_t* keys_in, uint64_t* keys_out, uint32_t n,
                    hipStream_t s);
hipError_t scan_u32_to_u64(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint64_t* out, uint32_t n,
                           hipStream_t s);
// inflate phase A in two launches: the first DEFLATE block's header + tables
// of every block of a chunk (k_huff_tables), then the decode reading them
// (round 0: the header at each block's start; round r > 0: where decode
// round r-1 left the block kHuffPending)
hipError_t launch_huff_tables(const uint8_t* file, const BlockInfo* blocks, uint32_t b0, uint32_t nb,
                              uint8_t* tables, HuffTableInfo* tinfo, const HuffOut* hout, uint32_t round,
                              hipStream_t s);
// (defer: stop a block before its next DEFLATE header, kHuffPending, for
// the next round; the last round decodes every remaining header inline)
hipError_t launch_inflate_huff_prebuilt(const uint8_t* file, const BlockInfo* blocks, uint32_t b0, uint32_t nb,
                                        uint64_t chunk_ustart, uint32_t* tokens, HuffOut* hout,
                                        const uint8_t* tables, const HuffTableInfo* tinfo, uint32_t round,
                                        uint32_t defer, hipStream_t s);
hipError_t launch_inflate_lz77(const BlockInfo* blocks, uint32_t b0, uint32_t nb, uint64_t chunk_ustart,
                               const uint32_t* tokens, const HuffOut* hout, uint8_t* u, hipStream_t s);
hipError_t launch_chain(const ChainArgs& a, int mode, int stage, hipStream_t s);
// a.cnt[i] = the records block i's list holds (0 off the chain): scanned into
// a.base, the offsets launch_rec_check_out writes at
hipError_t launch_list_counts(const ChainArgs& a, hipStream_t s);
// the record rules, long-cigar validation and output of the listed records
// (k_rec_check_out): cnt / err / need per block, outputs at a.base[i] (the
// scanned list counts), a.fuse_bad / a.fuse_flags as documented there; cap =
// the rec_pos / rec_voff / column capacity
hipError_t launch_rec_check_out(const ChainArgs& a, int mode, bool decode, const Columns& col, uint64_t cap,
                                hipStream_t s);
constexpr int kFusedBadShift = 40;
hipError_t link_scan_bytes(uint32_t nb, size_t* bytes);
hipError_t launch_rec_decode(const uint8_t* u, const uint64_t* rec_pos, uint64_t n, const Columns& col,
                             hipStream_t s);
hipError_t launch_first_error_hout(const HuffOut* hout, uint32_t b0, uint32_t nb, uint32_t* first, hipStream_t s);
hipError_t launch_records_after(const uint32_t* cnt, uint32_t nb, uint32_t k, uint32_t* flag, hipStream_t s);
hipError_t launch_first_error_i32(const int32_t* err, uint32_t nb, uint32_t* first, hipStream_t s);
hipError_t launch_truncate_counts(uint32_t* cnt, uint32_t nb, const uint32_t* cut, hipStream_t s);
// .splitting-bai entries of records with global ordinals o0 .. o0+n-1
// (ordinals k*g - 1): ent[j] for the j-th such ordinal of the span
hipError_t launch_sbi_emit(const uint64_t* voff, uint64_t n, uint32_t g, uint64_t o0, uint64_t* ent, hipStream_t s);
// *out = the chain successor of the last of n records (p0 when n == 0)
// gate_* (optional): a speculative launch, skipped on the device unless
// *gate_bad == ~0 and *gate_need <= gate_e_inf (k_rec_check_out's verdict)
hipError_t launch_next_pos(const uint8_t* u, const uint64_t* rec_pos, uint64_t n, uint64_t p0, int mode,
                           uint64_t* out, hipStream_t s, const unsigned long long* gate_bad = nullptr,
                           const unsigned long long* gate_need = nullptr, uint64_t gate_e_inf = 0);
// drop-in batches: records [0, n) of a decoded span -> an export slot
// (ColLayout with rec_pos; positions rebased by base, dst_pos[n] = nbytes);
// m > 0: also batch-major column blocks of m records at `packed`
// (k_export_records)
hipError_t launch_export_records(const Columns& src, const uint64_t* src_pos, const Columns& dst, uint64_t* dst_pos,
                                 uint64_t n, uint64_t base, uint64_t nbytes, uint8_t* packed, uint64_t m,
                                 hipStream_t s);
// n bytes device -> page-locked host by a kernel (no copy engine)
hipError_t launch_readback(void* dst, const void* src, uint64_t n, hipStream_t s);
// dst <- the rests of a span's records [0, n) back to back (record i's at
// rest_off[i] - p0 - 36 (i + 1)); u = the stream rest_off indexes; dst holds
// the rests' total + 16 bytes, u is readable 32 bytes past the last rest
hipError_t launch_pack_rests(const uint8_t* u, const uint64_t* rest_off, const uint32_t* rest_len, uint64_t n,
                             uint64_t p0, uint8_t* dst, hipStream_t s);
// dst[i] <- *src[i], i < n <= kGatherMax (dst: page-locked host or device)
constexpr int kGatherMax = 8;
hipError_t launch_gather_u64(uint64_t* dst, const uint64_t* const* src, int n, hipStream_t s);
// out[0] ^= xor of keys (if keys), out[1] += sum of voffs, out[2..3] += the
// order-sensitive key / voff digests (see k_digest)
hipError_t launch_digest(const int64_t* keys, const uint64_t* voffs, uint64_t n, uint64_t* out, hipStream_t s);
// keys deferred by decode_record (rest > kLongHash bytes): one wave per record
hipError_t launch_long_hash(const uint8_t* u, const uint64_t* rec_pos, const Columns& col, hipStream_t s,
                            const unsigned long long* gate_bad = nullptr, const unsigned long long* gate_need = nullptr,
                            uint64_t gate_e_inf = 0);
// SAMRecordWritable.write of a span's records: u[p0, p0+nbytes) -> dst
// (16 B-aligned, room for nbytes rounded up to 16) + bin patches (refID < 0)
hipError_t launch_wr_encode(const uint8_t* u, uint64_t p0, uint64_t nbytes, const uint64_t* rec_pos,
                            const int32_t* ref_id, const uint16_t* bin, uint64_t n, uint8_t* dst, hipStream_t s);
// SAMRecordWritable.readFields of n framed values; *bad = min((i << 8) | status)
hipError_t launch_wr_decode(const uint8_t* buf, uint64_t len, const uint64_t* offs, uint64_t n, const Columns& col,
                            uint64_t* rec_pos, unsigned long long* bad, hipStream_t s);

}  // namespace hbam
