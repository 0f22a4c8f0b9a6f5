// hbam_host.cpp -- C++ mirror of org.seqdoop.hadoop_bam's BAM read path
// classes on top of the gfx950 pipeline.  Host code here plans, validates
// headers and copies results; every per-record / per-byte loop of the hot path
// runs in hbam_kernels.hip.
#include "hbam_host.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

namespace hadoop_bam {

using hbam::kErrArg;
using hbam::kErrDevice;
using hbam::kErrFormat;
using hbam::kErrIO;
using hbam::kErrState;
using hbam::kErrTrunc;
using hbam::kOk;

// ---------------------------------------------------------------------------
// BamFile
// ---------------------------------------------------------------------------
int BamFile::open(const uint8_t* data, uint64_t len, int device, bool parse_header, bool check_crc,
                  std::unique_ptr<BamFile>* out, std::string* err) {
  (void)check_crc;  // CRC checking is opt-in in htsjdk's reader (off by default)
  std::unique_ptr<BamFile> f(new BamFile());
  f->file_.assign(data, data + len);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
    *err = "no HIP device " + std::to_string(device) + " (libhbam has no CPU path)";
    return kErrDevice;
  }
  f->pipe_.reset(new hbam::Pipeline(device));
  if (!f->pipe_->error().empty()) {
    *err = f->pipe_->error();
    return kErrDevice;
  }
  int rc = f->pipe_->load(f->file_.data(), len, 0);
  if (rc == kOk) rc = f->pipe_->locate();
  if (rc != kOk) {
    *err = f->pipe_->error();
    return rc;
  }
  if (parse_header) {
    rc = f->parse_header();
    if (rc != kOk) {
      *err = f->err_;
      return rc;
    }
  }
  *out = std::move(f);
  return kOk;
}

namespace {
// Sequential reader over the GPU-inflated stream (header parsing only).
struct StreamCursor {
  hbam::Pipeline& p;
  uint64_t pos = 0;
  std::vector<uint8_t> buf;
  uint64_t buf_pos = 0;
  explicit StreamCursor(hbam::Pipeline& pp) : p(pp) {}
  // returns bytes available (<= n) at pos, copied into dst
  int read(uint8_t* dst, uint64_t n, uint64_t* got) {
    *got = 0;
    while (*got < n) {
      if (pos >= buf_pos + buf.size() || pos < buf_pos) {
        uint64_t want = std::max<uint64_t>(n - *got, 1 << 20);
        int rc = p.read_stream(pos, want, &buf);
        if (rc != kOk) return rc;
        buf_pos = pos;
        if (buf.empty()) return kOk;
      }
      uint64_t k = std::min<uint64_t>(n - *got, buf_pos + buf.size() - pos);
      memcpy(dst + *got, buf.data() + (pos - buf_pos), k);
      *got += k;
      pos += k;
    }
    return kOk;
  }
};

int32_t rd_i32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}
}  // namespace

// [htsjdk] BAMFileReader.readHeader: magic, l_text, text, n_ref, refs; text
// @SQ lines, when present, must agree with the binary dictionary.
int BamFile::parse_header() {
  StreamCursor c(*pipe_);
  uint8_t b4[4];
  uint64_t got;
  int rc;
  if ((rc = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return rc; }
  if (got < 4 || memcmp(b4, "BAM\1", 4) != 0) { err_ = "Invalid BAM file header"; return kErrIO; }
  if ((rc = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return rc; }
  if (got < 4) { err_ = "Premature EOF in BAM header"; return kErrTrunc; }
  const int32_t l_text = rd_i32(b4);
  if (l_text < 0) { err_ = "Invalid BAM header: negative SAM header length " + std::to_string(l_text); return kErrIO; }
  text_.assign((size_t)l_text, '\0');
  if ((rc = c.read(reinterpret_cast<uint8_t*>(&text_[0]), (uint64_t)l_text, &got)) != kOk) { err_ = pipe_->error(); return rc; }
  if (got < (uint64_t)l_text) { err_ = "Premature EOF in BAM header text"; return kErrTrunc; }
  if ((rc = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return rc; }
  if (got < 4) { err_ = "Invalid BAM header: too short, no reference sequence count"; return kErrTrunc; }
  const int32_t n_ref = rd_i32(b4);
  if (n_ref < 0) { err_ = "Invalid BAM header: negative reference count"; return kErrIO; }
  for (int32_t i = 0; i < n_ref; ++i) {
    if ((rc = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return rc; }
    if (got < 4) { err_ = "Invalid reference list: EOF before reference " + std::to_string(i + 1); return kErrTrunc; }
    const int32_t l_name = rd_i32(b4);
    if (l_name < 0) { err_ = "negative reference name length"; return kErrIO; }
    std::string name((size_t)l_name, '\0');
    if ((rc = c.read(reinterpret_cast<uint8_t*>(&name[0]), (uint64_t)l_name, &got)) != kOk) { err_ = pipe_->error(); return rc; }
    if (got < (uint64_t)l_name) { err_ = "Premature EOF in reference name"; return kErrTrunc; }
    if (!name.empty() && name.back() == '\0') name.pop_back();
    if ((rc = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return rc; }
    if (got < 4) { err_ = "Premature EOF in reference length"; return kErrTrunc; }
    ref_names_.push_back(name);
    ref_lens_.push_back(rd_i32(b4));
  }
  n_ref_ = n_ref;
  header_end_ = c.pos;
  // text @SQ lines vs binary dictionary
  std::vector<std::pair<std::string, int64_t>> sq;
  size_t s = 0;
  while (s < text_.size()) {
    size_t e = text_.find('\n', s);
    if (e == std::string::npos) e = text_.size();
    if (text_.compare(s, 3, "@SQ") == 0) {
      std::string sn;
      int64_t ln = -1;
      size_t f = s;
      while (f < e) {
        size_t t = text_.find('\t', f);
        if (t == std::string::npos || t > e) t = e;
        if (text_.compare(f, 3, "SN:") == 0) sn = text_.substr(f + 3, t - f - 3);
        if (text_.compare(f, 3, "LN:") == 0) ln = strtoll(text_.c_str() + f + 3, nullptr, 10);
        f = t + 1;
      }
      sq.emplace_back(sn, ln);
    }
    s = e + 1;
  }
  if (!sq.empty()) {
    if ((int32_t)sq.size() != n_ref) {
      err_ = "Number of sequences in text header (" + std::to_string(sq.size()) +
             ") != number of sequences in binary header (" + std::to_string(n_ref) + ")";
      return kErrFormat;
    }
    for (int32_t i = 0; i < n_ref; ++i) {
      if (sq[i].first != ref_names_[i] || sq[i].second != ref_lens_[i]) {
        err_ = "Sequence " + std::to_string(i) + " in text header does not match binary header";
        return kErrFormat;
      }
    }
  }
  pipe_->set_n_ref(n_ref_);
  first_voff_ = pipe_->voff_of(header_end_);
  return kOk;
}

// ---------------------------------------------------------------------------
// SplittingBAMIndex
// ---------------------------------------------------------------------------
int SplittingBAMIndex::readIndex(const uint8_t* d, uint64_t len, std::string* err) {
  offsets_.clear();
  int64_t prev = -1;
  for (uint64_t k = 0; k + 8 <= len; k += 8) {
    uint64_t cur = 0;
    for (int i = 0; i < 8; ++i) cur = (cur << 8) | d[k + i];
    if (prev > (int64_t)cur) {
      char buf[128];
      snprintf(buf, sizeof buf, "Invalid splitting BAM index; offsets not in order: %#llx > %#llx",
               (unsigned long long)prev, (unsigned long long)cur);
      *err = buf;
      return kErrIO;
    }
    prev = (int64_t)cur;
    offsets_.insert(cur);
  }
  if (offsets_.empty()) {
    *err = "Invalid splitting BAM index: should contain at least the file size";
    return kErrIO;
  }
  return kOk;
}

bool SplittingBAMIndex::prevAlignment(uint64_t filePos, uint64_t* out) const {
  auto it = offsets_.upper_bound(filePos << 16);  // floor
  if (it == offsets_.begin()) return false;
  *out = *std::prev(it);
  return true;
}

bool SplittingBAMIndex::nextAlignment(uint64_t filePos, uint64_t* out) const {
  auto it = offsets_.upper_bound(filePos << 16);  // strictly higher
  if (it == offsets_.end()) return false;
  *out = *it;
  return true;
}

// ---------------------------------------------------------------------------
// SplittingBAMIndexer
// ---------------------------------------------------------------------------
static void put_be64(std::vector<uint8_t>* o, uint64_t v) {
  for (int i = 0; i < 8; ++i) o->push_back((uint8_t)(v >> (56 - 8 * i)));
}

int SplittingBAMIndexer::index(BamFile& f, int32_t g, std::vector<uint8_t>* out) {
  out->clear();
  if (g <= 0) {
    f.error() = "Granularity must be a positive integer";
    return kErrArg;
  }
  SpanDev span;
  // the chain starts at the header end (skipToAlignmentList :292-328)
  int rc = f.pipe().decode_span(f.first_record_voff(), ~0ull, hbam::kIndexer, false, &span);
  if (rc != kOk) {
    f.error() = f.pipe().error();
    return rc;
  }
  if (span.status != kOk) {
    f.error() = span.error;
    return span.status;
  }
  std::vector<uint64_t> ent;
  rc = f.pipe().splitting_entries(span, (uint32_t)g, &ent);
  if (rc != kOk) {
    f.error() = f.pipe().error();
    return rc;
  }
  out->reserve(8 * (ent.size() + 2));
  put_be64(out, f.first_record_voff());       // :262-264
  for (uint64_t v : ent) put_be64(out, v);     // :273-277
  put_be64(out, f.file_size() << 16);          // :286
  return kOk;
}

void SplittingBAMIndexer::processAlignment(uint64_t voff) {
  if (count_ == 0 || (count_ + 1) % (uint64_t)granularity_ == 0) writeVirtualOffset(voff);
  count_++;
}
void SplittingBAMIndexer::writeVirtualOffset(uint64_t v) { put_be64(&out_, v); }
void SplittingBAMIndexer::finish(uint64_t inputSize) { writeVirtualOffset(inputSize << 16); }

// ---------------------------------------------------------------------------
// BAMSplitGuesser (GPU batch; see hbam_guess.hip)
// ---------------------------------------------------------------------------
int guess_batch(BamFile& f, const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                std::vector<uint64_t>* out, std::string* err);

int BAMSplitGuesser::guessNextBAMRecordStarts(const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                                              std::vector<uint64_t>* out) {
  return guess_batch(f_, begs, ends, out, &f_.error());
}

// ---------------------------------------------------------------------------
// BAMInputFormat
// ---------------------------------------------------------------------------
int BAMInputFormat::addIndexedSplits(BamFile& f, const std::vector<FileSplit>& splits, const SplittingBAMIndex& idx,
                                     std::vector<FileVirtualSplit>* out, bool* bad_index) {
  (void)f;
  *bad_index = false;
  if (idx.size() == 1) return kOk;  // :280-282 only the file size: no alignments
  std::vector<FileVirtualSplit> pot;
  for (size_t j = 0; j < splits.size(); ++j) {
    const uint64_t start = splits[j].start, end = start + splits[j].length;
    uint64_t bs = 0, be = 0;
    const bool hs = idx.nextAlignment(start, &bs);                         // :290
    bool he;
    if (j == splits.size() - 1) {
      he = idx.prevAlignment(end, &be);                                    // :299-300
      be |= 0xffff;
    } else {
      he = idx.nextAlignment(end, &be);                                    // :302
    }
    if (!hs || !he) {                                                      // :305-308
      *bad_index = true;
      return kOk;
    }
    FileVirtualSplit v;
    v.path = splits[j].path;
    v.vStart = bs;
    v.vEnd = be;
    pot.push_back(v);
  }
  out->insert(out->end(), pot.begin(), pot.end());
  return kOk;
}

int BAMInputFormat::addProbabilisticSplits(BamFile& f, const std::vector<FileSplit>& splits,
                                           std::vector<FileVirtualSplit>* out) {
  std::vector<uint64_t> begs, ends, guess;
  for (auto& s : splits) {
    begs.push_back(s.start);
    ends.push_back(s.start + s.length);
  }
  BAMSplitGuesser g(f);
  int rc = g.guessNextBAMRecordStarts(begs, ends, &guess);
  if (rc != kOk) return rc;
  int64_t prev = -1;
  for (size_t i = 0; i < splits.size(); ++i) {
    const uint64_t alignedBeg = guess[i];                 // :490
    const uint64_t alignedEnd = (ends[i] << 16) | 0xffff; // :495
    if (alignedBeg == ends[i]) {                          // :497-513
      if (prev < 0) {
        f.error() = "'" + splits[i].path + "': no reads in first split: bad BAM file or tiny split size?";
        return kErrIO;
      }
      (*out)[(size_t)prev].setEndVirtualOffset(alignedEnd);
    } else {
      FileVirtualSplit v;
      v.path = splits[i].path;
      v.vStart = alignedBeg;
      v.vEnd = alignedEnd;
      out->push_back(v);
      prev = (int64_t)out->size() - 1;
    }
  }
  return kOk;
}

int BAMInputFormat::getSplits(BamFile& f, const std::vector<FileSplit>& splits, const uint8_t* sbi,
                              uint64_t sbi_len, std::vector<FileVirtualSplit>* out) {
  out->clear();
  if (sbi) {
    SplittingBAMIndex idx;
    std::string err;
    if (idx.readIndex(sbi, sbi_len, &err) == kOk) {
      bool bad = false;
      int rc = addIndexedSplits(f, splits, idx, out, &bad);
      if (rc != kOk) return rc;
      if (!bad) return kOk;
      out->clear();  // "Index ... was not good. Generating probabilistic splits."
    }
    // readIndex IOException: getSplits' catch falls back to probabilistic splits (:245-257)
  }
  return addProbabilisticSplits(f, splits, out);
}

// ---------------------------------------------------------------------------
// BAMRecordReader
// ---------------------------------------------------------------------------
int fetch_span(hbam::Pipeline& p, const SpanDev& s, BAMRecordReader::Host* h, std::string* err) {
  const uint64_t n = s.n;
  auto cp = [&](auto& vec, const auto* src) -> int {
    vec.resize(n);
    if (n == 0) return kOk;
    if (hipMemcpyAsync(vec.data(), src, n * sizeof(vec[0]), hipMemcpyDeviceToHost, p.stream()) != hipSuccess) {
      *err = "hipMemcpy D2H failed";
      return kErrDevice;
    }
    return kOk;
  };
  const hbam::Columns& c = s.col;
  int rc = kOk;
  rc |= cp(h->ref_id, c.ref_id);
  rc |= cp(h->pos, c.pos);
  rc |= cp(h->l_seq, c.l_seq);
  rc |= cp(h->next_ref_id, c.next_ref_id);
  rc |= cp(h->next_pos, c.next_pos);
  rc |= cp(h->tlen, c.tlen);
  rc |= cp(h->l_read_name, c.l_read_name);
  rc |= cp(h->mapq, c.mapq);
  rc |= cp(h->bin, c.bin);
  rc |= cp(h->n_cigar, c.n_cigar);
  rc |= cp(h->flag, c.flag);
  rc |= cp(h->key, c.key);
  rc |= cp(h->voff, c.voff);
  rc |= cp(h->rest_off, c.rest_off);
  rc |= cp(h->rest_len, c.rest_len);
  if (rc != kOk) return kErrDevice;
  if (hipStreamSynchronize(p.stream()) != hipSuccess) {
    *err = "hipStreamSynchronize failed";
    return kErrDevice;
  }
  // inflated bytes of the span: [p0, end of the last record)
  uint64_t lo = s.p0, hi = s.p0;
  if (n) hi = h->rest_off[n - 1] + h->rest_len[n - 1];
  h->data.resize(hi - lo);
  if (hi > lo) {
    if (hipMemcpy(h->data.data(), (s.data ? s.data : p.d_u()) + lo, hi - lo, hipMemcpyDeviceToHost) != hipSuccess) {
      *err = "hipMemcpy D2H failed";
      return kErrDevice;
    }
  }
  for (uint64_t i = 0; i < n; ++i) h->rest_off[i] -= lo;
  return kOk;
}

int BAMRecordReader::initialize(BamFile& f, const FileVirtualSplit& split) {
  // :131-133 re-entrant initialize
  *this = BAMRecordReader();
  const uint64_t vs = split.getStartVirtualOffset();
  fileStart_ = vs >> 16;                     // :153
  virtualEnd_ = split.getEndVirtualOffset(); // :154
  SpanDev span;
  int rc = f.pipe().decode_span(vs, virtualEnd_, hbam::kReader, true, &span);
  if (rc != kOk) {
    err_ = f.pipe().error();
    status_ = rc;
    return rc;
  }
  rc = fetch_span(f.pipe(), span, &h_, &err_);
  if (rc != kOk) {
    status_ = rc;
    return rc;
  }
  n_ = span.n;
  status_ = span.status;
  if (status_ != kOk) err_ = span.error;
  return kOk;
}

bool BAMRecordReader::nextKeyValue() {
  if (started_) ++cur_;
  started_ = true;
  if (cur_ >= n_) return false;  // status() tells a clean end from an error
  view_.refID = h_.ref_id[cur_];
  view_.pos = h_.pos[cur_];
  view_.l_seq = h_.l_seq[cur_];
  view_.next_refID = h_.next_ref_id[cur_];
  view_.next_pos = h_.next_pos[cur_];
  view_.tlen = h_.tlen[cur_];
  view_.l_read_name = h_.l_read_name[cur_];
  view_.mapq = h_.mapq[cur_];
  view_.bin = h_.bin[cur_];
  view_.n_cigar = h_.n_cigar[cur_];
  view_.flag = h_.flag[cur_];
  view_.voff = h_.voff[cur_];
  view_.rest = h_.data.data() + h_.rest_off[cur_];
  view_.rest_len = h_.rest_len[cur_];
  lastVoff_ = view_.voff;
  return true;
}

float BAMRecordReader::getProgress() const {
  if (started_ && cur_ >= n_) return 1.0f;
  const uint64_t filePos = lastVoff_ >> 16, fileEnd = virtualEnd_ >> 16;
  if (filePos < fileStart_) return 0.0f;
  return (float)(filePos - fileStart_) / (float)(fileEnd - fileStart_ + 1);
}

// ---------------------------------------------------------------------------
int64_t murmurhash3(const uint8_t* key, uint64_t len64, int32_t seed) {
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto fmix = [](uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
  };
  auto rd64 = [](const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
  };
  const int32_t len = (int32_t)len64;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  uint64_t h1 = (uint64_t)(int64_t)seed, h2 = h1;
  const int32_t nb = len / 16;
  for (int32_t i = 0; i < nb; ++i) {
    uint64_t k1 = rd64(key + 16 * i), k2 = rd64(key + 16 * i + 8);
    k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = (h2 << 31) | (h1 >> 33); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* t = key + 16 * nb;
  const int r = len & 15;
  uint64_t k1 = 0, k2 = 0;
  for (int j = r - 1; j >= 8; --j) k2 = (k2 << 8) | t[j];
  if (r > 8) { k2 *= c2; k2 = rotl(k2, 33); k2 *= c1; h2 ^= k2; }
  for (int j = std::min(r, 8) - 1; j >= 0; --j) k1 = (k1 << 8) | t[j];
  if (r > 0) { k1 *= c1; k1 = rotl(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= (uint64_t)(int64_t)len;
  h2 ^= (uint64_t)(int64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix(h1);
  h2 = fmix(h2);
  h1 += h2;
  return (int64_t)h1;
}

}  // namespace hadoop_bam
