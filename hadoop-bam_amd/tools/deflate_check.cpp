// deflate_check.cpp -- test tool (not product): the hbam_deflate.h
// restatement compiled for the host, byte-compared with system zlib 1.2.11
// (deflateInit2(level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY)) over block
// sequences, in both Deflater lifecycles:
//   reuse: one stream, deflateReset per block ([htsjdk]
//          BlockCompressedOutputStream: deflater.reset() per block)
//   fresh: deflateInit2 per block (htslib bgzf, tools/gen_synth_bam.c)
// Usage: deflate_check [file ...]   (files are cut into 65498/65280/... blocks;
// without files: built-in random / repetitive / text / short-block cases).
// Prints one line per case and "ALL OK" when everything matched.
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../csrc/hbam_deflate.h"

using namespace hbam::dfl;

static Tables g_t;

static int run_case(const char* name, const std::vector<uint8_t>& data, const std::vector<uint32_t>& sizes, int level,
                    bool fresh) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 1;
  std::unique_ptr<Arena> a(new Arena());
  memset(a.get(), 0, sizeof(Arena));
  std::vector<uint8_t> zo(140000), mo(140000);
  uint64_t off = 0;
  int bad = 0;
  size_t bi = 0;
  for (uint32_t len : sizes) {
    const uint8_t* in = data.data() + off;
    if (fresh) {
      deflateEnd(&z);
      deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    } else {
      deflateReset(&z);
    }
    z.next_in = const_cast<uint8_t*>(in);
    z.avail_in = len;
    z.next_out = zo.data();
    z.avail_out = (uInt)zo.size();
    int rc = deflate(&z, Z_FINISH);
    const uint32_t zn = (uint32_t)(zo.size() - z.avail_out);
    bool ovf = false;
    const uint32_t mn = deflate_block(a.get(), &g_t, level, in, len, mo.data(), (uint32_t)mo.size(), &ovf);
    if (rc != Z_STREAM_END || zn != mn || memcmp(zo.data(), mo.data(), zn) != 0) {
      uint32_t k = 0;
      while (k < zn && k < mn && zo[k] == mo[k]) ++k;
      if (bad < 5)
        printf("  MISMATCH %s level %d %s block %zu len %u: zlib %u bytes, ours %u, first diff at %u\n", name, level,
               fresh ? "fresh" : "reuse", bi, len, zn, mn, k);
      ++bad;
    }
    off += len;
    ++bi;
  }
  deflateEnd(&z);
  printf("%s %s level %d %s: %zu blocks, %d mismatches\n", bad ? "FAIL" : "ok  ", name, level,
         fresh ? "fresh" : "reuse", sizes.size(), bad);
  return bad;
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}

static std::vector<uint32_t> cut(uint64_t total, uint32_t bs) {
  std::vector<uint32_t> s;
  while (total) {
    uint32_t l = (uint32_t)(total < bs ? total : bs);
    s.push_back(l);
    total -= l;
  }
  return s;
}

int main(int argc, char** argv) {
  build_tables(&g_t);
  int bad = 0;
  std::vector<std::pair<std::string, std::vector<uint8_t>>> inputs;
  for (int i = 1; i < argc; ++i) {
    FILE* f = fopen(argv[i], "rb");
    if (!f) return 2;
    std::vector<uint8_t> b;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    inputs.push_back({argv[i], b});
  }
  if (inputs.empty()) {
    std::vector<uint8_t> r(700000);  // incompressible: stored blocks, sym-buffer flushes
    for (auto& c : r) c = (uint8_t)rnd();
    inputs.push_back({"random", r});
    std::vector<uint8_t> lowent(700000);  // small alphabet: many matches + literals
    for (auto& c : lowent) c = "ACGT"[rnd() & 3];
    inputs.push_back({"acgt", lowent});
    std::vector<uint8_t> rep(700000);  // long runs: max-length matches, dist 1
    for (size_t i = 0; i < rep.size(); ++i) rep[i] = (uint8_t)((i / 5000) & 0xff);
    inputs.push_back({"runs", rep});
    std::vector<uint8_t> txt;  // SAM-ish text with quality-like noise
    while (txt.size() < 900000) {
      char line[512];
      int q = snprintf(line, sizeof line, "SYN:1:%u:%u:%u\t%u\tchr%u\t%u\t60\t150M\t=\t%u\t0\t", rnd() % 100,
                       rnd() % 30000, rnd() % 30000, rnd() % 4 * 16, rnd() % 22 + 1, rnd() % 100000000,
                       rnd() % 100000000);
      txt.insert(txt.end(), line, line + q);
      for (int k = 0; k < 150; ++k) txt.push_back("ACGTN"[rnd() % 5 == 4 ? 4 : rnd() & 3]);
      txt.push_back('\t');
      for (int k = 0; k < 150; ++k) txt.push_back((uint8_t)(33 + 2 + (rnd() % 40 < 30 ? 35 + rnd() % 6 : rnd() % 40)));
      txt.push_back('\n');
    }
    inputs.push_back({"samtext", txt});
  }
  if (argc == 1) {
    // payloads past the slide threshold over a 2-letter alphabet: matches run
    // into the window bytes past the data end after the slide
    std::vector<uint8_t> ab(4000000);
    for (auto& c : ab) c = "AC"[rnd() & 1];
    std::vector<uint32_t> sz;
    uint64_t tot = 0;
    while (tot + 65536 < ab.size()) {
      uint32_t l = 65274 + rnd() % 263;
      sz.push_back(l);
      tot += l;
    }
    for (int level : {1, 5, 9}) {
      bad += run_case("ac-sliders", ab, sz, level, false);
      bad += run_case("ac-sliders", ab, sz, level, true);
    }
  }
  for (auto& in : inputs) {
    const std::vector<uint8_t>& d = in.second;
    for (int level : {5}) {
      for (uint32_t bs : {65498u, 65280u}) {
        bad += run_case(in.first.c_str(), d, cut(d.size(), bs), level, false);
        bad += run_case(in.first.c_str(), d, cut(d.size(), bs), level, true);
      }
    }
    // ragged sizes incl. 0, 1, 2, 3, around the slide threshold and 65536
    std::vector<uint32_t> rag = {0, 1, 2, 3, 4, 257, 258, 259, 65273, 65274, 65275, 65536, 1000, 65498, 300, 40000};
    uint64_t tot = 0;
    for (uint32_t v : rag) tot += v;
    if (d.size() >= tot) {
      for (int level : {1, 3, 4, 5, 6, 9}) {
        bad += run_case((in.first + "/ragged").c_str(), d, rag, level, false);
        bad += run_case((in.first + "/ragged").c_str(), d, rag, level, true);
      }
    }
    for (int level : {1, 2, 3, 4, 6, 7, 8, 9}) bad += run_case(in.first.c_str(), d, cut(d.size() < 400000 ? d.size() : 400000, 65498), level, false);
  }
  printf(bad ? "FAILED (%d)\n" : "ALL OK\n", bad);
  return bad ? 1 : 0;
}
