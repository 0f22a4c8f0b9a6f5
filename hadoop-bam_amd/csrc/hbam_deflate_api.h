// hbam_deflate_api.h -- host side of the GPU BGZF compressor (hbam_deflate.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace hbam {
namespace dfl {
struct Tables;
struct Arena;
}  // namespace dfl

// [htsjdk] BlockCompressedOutputStream over a device-resident payload stream:
// block b = d_in[ustart[b], ustart[b] + lens[b]).  Output (BGZF file bytes,
// optionally with the 28-byte EOF terminator) stays on the device.
class BgzfCompressor {
 public:
  explicit BgzfCompressor(int device);
  ~BgzfCompressor();
  BgzfCompressor(const BgzfCompressor&) = delete;
  BgzfCompressor& operator=(const BgzfCompressor&) = delete;

  // Status codes as include/hbam.h; *ms = HIP-event time of the whole call.
  int compress(const uint8_t* d_in, const std::vector<uint64_t>& ustart, const std::vector<uint32_t>& lens, int level,
               bool eof, hipStream_t s, float* ms);
  const uint8_t* d_out() const { return out_; }
  uint64_t out_len() const { return out_len_; }
  uint64_t fallbacks() const { return fallbacks_; }  // blocks written by the level-0 fallback
  const std::string& error() const { return err_; }

 private:
  int device_;
  std::string err_;
  dfl::Tables* tables_ = nullptr;
  dfl::Arena* arenas_ = nullptr;
  uint8_t *slots_ = nullptr, *ovf_ = nullptr, *out_ = nullptr;
  uint32_t *csize_ = nullptr, *crc_ = nullptr, *lens_ = nullptr;
  uint32_t* crc_tab_ = nullptr;  // k_dfl_crc constants: slice-by-8 tables + combine multipliers
  uint64_t *offs_ = nullptr, *ustart_ = nullptr;
  size_t arenas_n_ = 0, slots_n_ = 0, csize_n_ = 0, ovf_n_ = 0, crc_n_ = 0, offs_n_ = 0, out_n_ = 0, ustart_n_ = 0,
         lens_n_ = 0;
  uint64_t out_len_ = 0, fallbacks_ = 0;
};

}  // namespace hbam
