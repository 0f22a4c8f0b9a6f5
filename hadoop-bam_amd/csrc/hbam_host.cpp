// hbam_host.cpp -- C++ mirror of org.seqdoop.hadoop_bam's BAM read path
// classes on top of the gfx950 pipeline.  Host code here plans windows,
// parses the header and copies results; every per-record / per-byte loop of
// the hot path runs in hbam_kernels.hip.
#include "hbam_mem.h"
#include "hbam_host.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>

namespace hadoop_bam {

using hbam::BlockInfo;
using hbam::kErrArg;
using hbam::kErrDevice;
using hbam::kErrFormat;
using hbam::kErrIO;
using hbam::kErrNoMem;
using hbam::kErrState;
using hbam::kErrTrunc;
using hbam::kOk;

// ---------------------------------------------------------------------------
// PinnedVec / Source
// ---------------------------------------------------------------------------
template <typename T>
bool PinnedVec<T>::resize(size_t n) {
  if (n <= cap_) {
    n_ = n;
    return true;
  }
  size_t c = std::max(n, cap_ + cap_ / 2);
  void* q = nullptr;
  size_t got = 0;
  if (hbam::pinned_alloc(&q, std::max<size_t>(c, 1) * sizeof(T), &got) != hipSuccess) return false;
  if (p_ && n_) memcpy(q, p_, n_ * sizeof(T));
  if (p_) hbam::pinned_free(p_, cap_ * sizeof(T));
  p_ = static_cast<T*>(q);
  cap_ = got / sizeof(T);
  n_ = n;
  return true;
}
template <typename T>
void PinnedVec<T>::release() {
  if (p_) hbam::pinned_free(p_, cap_ * sizeof(T));
  p_ = nullptr;
  n_ = cap_ = 0;
}
template class PinnedVec<int32_t>;
template class PinnedVec<uint8_t>;
template class PinnedVec<uint16_t>;
template class PinnedVec<int64_t>;
template class PinnedVec<uint64_t>;
template class PinnedVec<uint32_t>;

Source::~Source() {
  if (map) munmap(map, map_len);
  if (fd >= 0) ::close(fd);
}

// ---------------------------------------------------------------------------
// BamFile
// ---------------------------------------------------------------------------
int BamFile::open_memory(const uint8_t* data, uint64_t len, const OpenOptions& o, std::unique_ptr<BamFile>* out,
                         std::string* err) {
  std::unique_ptr<BamFile> f(new BamFile());
  f->src_.owned.assign(data, data + len);
  static const uint8_t empty = 0;
  f->src_.host.mem = len ? f->src_.owned.data() : &empty;
  f->src_.host.size = len;
  f->src_.size = len;
  int rc = f->init(o, err);
  if (rc == kOk) *out = std::move(f);
  return rc;
}

int BamFile::open_path(const char* path, const OpenOptions& o, std::unique_ptr<BamFile>* out, std::string* err) {
  std::unique_ptr<BamFile> f(new BamFile());
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) {
    *err = std::string("cannot open ") + path;
    return kErrIO;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    *err = std::string("cannot stat ") + path;
    return kErrIO;
  }
  f->src_.size = (uint64_t)st.st_size;
  // pages are read only when a window copies them (WrapSeekable seeks); the
  // fd stays open for the length check before each read (HostSource)
  f->src_.fd = fd;
  f->src_.host.fd = fd;
  f->src_.host.size = (uint64_t)st.st_size;
  if (st.st_size > 0) {
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      *err = std::string("cannot map ") + path;
      return kErrIO;  // (f closes fd)
    }
    f->src_.map = m;
    f->src_.map_len = (size_t)st.st_size;
    f->src_.host.mem = static_cast<const uint8_t*>(m);
  } else {
    static const uint8_t empty = 0;
    f->src_.host.mem = &empty;
  }
  int rc = f->init(o, err);
  if (rc == kOk) *out = std::move(f);
  return rc;
}

int BamFile::open_reader(uint64_t size, hbam::HostSource::ReadFn fn, void* user, const OpenOptions& o,
                         std::unique_ptr<BamFile>* out, std::string* err) {
  if (!fn) {
    *err = "no reader";
    return kErrArg;
  }
  std::unique_ptr<BamFile> f(new BamFile());
  f->src_.size = size;
  f->src_.host.read_fn = fn;
  f->src_.host.user = user;
  f->src_.host.size = size;
  f->src_.host.concurrent = o.parallel_reads;
  int rc = f->init(o, err);
  if (rc == kOk) *out = std::move(f);
  return rc;
}

int BamFile::open_device_copy(const uint8_t* data, uint64_t len, const OpenOptions& o, std::unique_ptr<BamFile>* out,
                              std::string* err) {
  std::unique_ptr<BamFile> f(new BamFile());
  f->src_.size = len;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= o.device || o.device < 0) {
    *err = "no HIP device " + std::to_string(o.device) + " (libhbam has no CPU path)";
    return kErrDevice;
  }
  if (hipSetDevice(o.device) != hipSuccess || f->src_.dev.reserve(len + hbam::kFilePad) != hipSuccess ||
      (len && hipMemcpy(f->src_.dev.p, data, len, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemset(f->src_.dev.p + len, 0, hbam::kFilePad) != hipSuccess) {
    *err = "cannot make the file resident in HBM";
    return kErrDevice;
  }
  f->src_.dev_lo = 0;
  f->src_.dev_hi = len;
  f->src_.bytes_read = len;
  int rc = f->init(o, err);
  if (rc == kOk) *out = std::move(f);
  return rc;
}

int BamFile::init(const OpenOptions& o, std::string* err) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= o.device || o.device < 0) {
    *err = "no HIP device " + std::to_string(o.device) + " (libhbam has no CPU path)";
    return kErrDevice;
  }
  pipe_.reset(new hbam::Pipeline(o.device));
  if (!pipe_->error().empty()) {
    *err = pipe_->error();
    return kErrDevice;
  }
  src_.dev.owner = &pipe_->streams();  // kernels read the resident copy on the pipeline's streams
  pipe_->set_stringency(o.stringency);
  set_window_bytes(o.window_bytes ? o.window_bytes : kDefaultWindowBytes);
  window_explicit_ = o.window_bytes != 0;
  int rc;
  if (o.parse_header) {
    rc = parse_header();
  } else {  // plain BGZF: the first window's framing is checked at open
    rc = load_window(0, std::min<uint64_t>(src_.size, window_bytes_));
  }
  if (rc != kOk) *err = err_;
  return rc;
}

int BamFile::prefetch(uint64_t lo, uint64_t hi) {
  hi = std::min(hi, src_.size);
  if (lo >= hi) return kOk;
  if (!src_.host.valid()) {
    err_ = "prefetch needs a host copy of the file";
    return kErrState;
  }
  // byte lo lands at dev.p + lo % 16: file offsets keep their 16 B alignment
  // on the device, which the kernels' aligned loads assume
  if (hipSetDevice(pipe_->device()) != hipSuccess || src_.dev.reserve(hi - lo + 16 + hbam::kFilePad) != hipSuccess) {
    err_ = "prefetch: HBM allocation failed";
    return kErrDevice;
  }
  uint8_t* at = src_.dev.p + (lo & 15);
  src_.dev_lo = src_.dev_hi = 0;  // nothing resident until the copy succeeds
  win_lo_ = ~0ull;
  if (int rc = pipe_->copy_from_host(at, src_.host, lo, hi - lo)) {
    err_ = "prefetch: " + pipe_->error();
    return rc;
  }
  if (hipMemset(at + (hi - lo), 0, hbam::kFilePad) != hipSuccess) {
    err_ = "prefetch: HIP copy failed";
    return kErrDevice;
  }
  src_.dev_lo = lo;
  src_.dev_hi = hi;
  src_.bytes_read += hi - lo;
  win_lo_ = ~0ull;  // the loaded window may point at the old copy
  return kOk;
}

namespace { void htrace(const char* what); }

int BamFile::load_window(uint64_t lo, uint64_t hi, bool free_start, bool host_only) {
  hi = std::min(hi, src_.size);
  if (hi < lo) hi = lo;
  const bool dev = !host_only && src_.dev.p && lo >= src_.dev_lo && lo < src_.dev_hi;
  if (dev) hi = std::min(hi, src_.dev_hi);
  if (lo == win_lo_ && hi == win_hi_ && free_start == win_free_) return kOk;  // already loaded and located
  win_lo_ = ~0ull;
  int rc;
  if (dev) {
    rc = pipe_->attach_device(src_.dev.p + (src_.dev_lo & 15) + (lo - src_.dev_lo), hi - lo, lo, hi == src_.size);
  } else {
    if (!src_.host.valid()) {
      err_ = "file bytes [" + std::to_string(lo) + ", " + std::to_string(hi) + ") are not resident in HBM";
      return kErrState;
    }
    uint64_t copied = 0;
    rc = pipe_->load(src_.host, hi - lo, lo, hi == src_.size, &copied);
    src_.bytes_read += copied;
    htrace(copied ? "window bytes copied to HBM" : "window bytes already in HBM");
  }
  if (rc == kOk) rc = pipe_->locate(free_start);
  if (rc != kOk) {
    err_ = pipe_->error();
    return rc;
  }
  win_lo_ = lo;
  win_hi_ = hi;
  win_free_ = free_start;
  return kOk;
}

namespace {
// Sequential reader over the current window's inflated stream (header parse).
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
// @SQ lines, when present, must agree with the binary dictionary.  Read from
// a window at the start of the file that grows until the header fits.
int BamFile::parse_header() {
  uint64_t w = std::min<uint64_t>(src_.size, std::min<uint64_t>(window_bytes_, 1ull << 20));
  for (;;) {
    int rc = load_window(0, w);
    if (rc != kOk) return rc;
    const bool whole = pipe_->at_eof();
    StreamCursor c(*pipe_);
    uint8_t b4[4];
    uint64_t got;
    auto more = [&](int code, const char* msg) {  // a short read in an open window: grow it
      if (!whole) return -1;
      err_ = msg;
      return code;
    };
    text_.clear();
    ref_names_.clear();
    ref_lens_.clear();
    rc = [&]() -> int {
      int r;
      if ((r = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return r; }
      if (got < 4) return more(kErrIO, "Invalid BAM file header");
      if (memcmp(b4, "BAM\1", 4) != 0) { err_ = "Invalid BAM file header"; return kErrIO; }
      if ((r = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return r; }
      if (got < 4) return more(kErrTrunc, "Premature EOF in BAM header");
      const int32_t l_text = rd_i32(b4);
      if (l_text < 0) { err_ = "Invalid BAM header: negative SAM header length " + std::to_string(l_text); return kErrIO; }
      text_.assign((size_t)l_text, '\0');
      if ((r = c.read(reinterpret_cast<uint8_t*>(&text_[0]), (uint64_t)l_text, &got)) != kOk) { err_ = pipe_->error(); return r; }
      if (got < (uint64_t)l_text) return more(kErrTrunc, "Premature EOF in BAM header text");
      if ((r = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return r; }
      if (got < 4) return more(kErrTrunc, "Invalid BAM header: too short, no reference sequence count");
      const int32_t n_ref = rd_i32(b4);
      if (n_ref < 0) { err_ = "Invalid BAM header: negative reference count"; return kErrIO; }
      for (int32_t i = 0; i < n_ref; ++i) {
        if ((r = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return r; }
        if (got < 4) return more(kErrTrunc, "Invalid reference list: EOF before reference");
        const int32_t l_name = rd_i32(b4);
        if (l_name < 0) { err_ = "negative reference name length"; return kErrIO; }
        std::string name((size_t)l_name, '\0');
        if ((r = c.read(reinterpret_cast<uint8_t*>(&name[0]), (uint64_t)l_name, &got)) != kOk) { err_ = pipe_->error(); return r; }
        if (got < (uint64_t)l_name) return more(kErrTrunc, "Premature EOF in reference name");
        if (!name.empty() && name.back() == '\0') name.pop_back();
        if ((r = c.read(b4, 4, &got)) != kOk) { err_ = pipe_->error(); return r; }
        if (got < 4) return more(kErrTrunc, "Premature EOF in reference length");
        ref_names_.push_back(name);
        ref_lens_.push_back(rd_i32(b4));
      }
      n_ref_ = n_ref;
      return kOk;
    }();
    if (rc == -1) {  // the header runs past this window
      if (w >= src_.size) return kErrTrunc;
      w = std::min<uint64_t>(src_.size, 2 * w);
      continue;
    }
    if (rc != kOk) return rc;
    const uint64_t header_end = c.pos;
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
      if ((int32_t)sq.size() != n_ref_) {
        err_ = "Number of sequences in text header (" + std::to_string(sq.size()) +
               ") != number of sequences in binary header (" + std::to_string(n_ref_) + ")";
        return kErrFormat;
      }
      for (int32_t i = 0; i < n_ref_; ++i) {
        if (sq[i].first != ref_names_[i] || sq[i].second != ref_lens_[i]) {
          err_ = "Sequence " + std::to_string(i) + " in text header does not match binary header";
          return kErrFormat;
        }
      }
    }
    pipe_->set_n_ref(n_ref_);
    rc = pipe_->set_ref_lengths(ref_lens_);
    if (rc != kOk) {
      err_ = pipe_->error();
      return rc;
    }
    first_voff_ = pipe_->voff_of(header_end);
    return kOk;
  }
}

namespace {
void htrace(const char* what) {  // HBAM_CURSOR_TRACE: developer timing lines on stderr
  static const bool t = getenv("HBAM_CURSOR_TRACE") != nullptr;
  if (!t) return;
  static auto last = std::chrono::steady_clock::now();
  const auto now = std::chrono::steady_clock::now();
  fprintf(stderr, "[step] +%.3f ms %s\n", std::chrono::duration<double, std::milli>(now - last).count(), what);
  last = now;
}
}  // namespace

int BamFile::decode_step(Carry from, uint64_t vend, hbam::ChainMode mode, bool decode, bool continuation,
                         Step* out, uint64_t window, uint64_t next_window) {
  htrace("decode_step");
  *out = Step();
  Carry c = from;
  uint64_t span_w = window ? std::max<uint64_t>(window, 1ull << 16) : window_bytes_;
  bool host_only = false, clamp = vend != ~0ull;
  for (int guard = 0; guard < 96; ++guard) {
    out->next = c;
    if (c.upos <= 0xffff && c.voff() >= vend) return kOk;  // the split ends here
    if (c.coff >= src_.size) return kOk;                    // past the last block: end of stream
    // a split ending at vend needs its last record's bytes, rarely more than
    // a block past vend: no need to copy a whole window beyond it
    uint64_t hi = c.coff + span_w;
    if (clamp) hi = std::min(hi, std::max((vend >> 16) + 0x20000, c.coff + 0x20000));
    int rc = load_window(c.coff, hi, false, host_only);
    if (rc != kOk) return rc;
    htrace("load_window + locate");
    hbam::Pipeline& p = *pipe_;
    // the split goes on past this window: start the next window's new bytes
    // on their way to HBM while this one decodes (Pipeline::stage)
    if (src_.host.valid() && win_hi_ < src_.size && (!clamp || win_hi_ < (vend >> 16) + 0x20000)) {
      // the next window starts at the record this one cannot finish (a few
      // blocks before win_hi_), so it ends up to that tail short of
      // win_hi_ + span_w: stage that much less, or the bytes past its end
      // would be copied again by the window after it
      // (next_window: the caller's next window is a different size)
      const uint64_t nw = next_window ? std::max<uint64_t>(next_window, 1ull << 16) : span_w;
      const uint64_t s_lo = win_hi_;
      const uint64_t tail = std::min<uint64_t>(nw / 2, 4 * 65536);
      uint64_t s_hi = std::min(src_.size, s_lo + nw - tail);
      if (clamp) s_hi = std::min(s_hi, std::max((vend >> 16) + 0x20000, s_lo));
      const bool resident = src_.dev.p && s_lo >= src_.dev_lo && s_hi <= src_.dev_hi;
      if (s_hi > s_lo && !resident) {
        rc = p.stage(src_.host, s_lo, s_hi);
        if (rc != kOk) {
          err_ = p.error();
          return rc;
        }
        if (s_lo != staged_lo_ || s_hi != staged_hi_) src_.bytes_read += s_hi - s_lo;
        staged_lo_ = s_lo;
        staged_hi_ = s_hi;
      }
    }
    const auto& B = p.blocks();
    if (B.empty()) {
      if (p.at_eof()) return kOk;  // no complete block left
      span_w *= 2;                 // a block longer than the window
      continue;
    }
    if (B[0].coff != c.coff || (!continuation && c.upos > B[0].isize)) {
      err_ = "Invalid file pointer: " + std::to_string(c.voff());
      return kErrIO;
    }
    // [htsjdk] an empty block right after an exhausted one reads as EOF
    if (continuation && c.upos == 0 && B[0].isize == 0) return kOk;
    const uint64_t p0 = c.upos;
    if (p0 > p.total_u() || (p0 == p.total_u() && !p.at_eof())) {
      // the indexer skipped past this window (a record longer than it)
      if (p.at_eof()) {
        out->status = kErrIO;
        out->error = "Skip failed: record runs past the end of the file";
        return kOk;
      }
      c = Carry{p.window_end(), p0 - p.total_u()};
      continuation = true;
      continue;
    }
    SpanDev s;
    htrace("stage started");
    rc = p.decode_span_pos(p0, vend, mode, decode, &s);
    htrace("decode_span_pos");
    if (rc != kOk) {
      err_ = p.error();
      return rc;
    }
    if (s.status == kOk && s.n == 0 && s.next_pos == p0 && p0 < s.q_end && !p.at_eof()) {
      // the first record does not end inside this window: a bigger one
      if (win_hi_ < std::min(src_.size, hi) && !host_only) host_only = true;  // clipped by the HBM-resident range
      else span_w = 2 * std::max(span_w, win_hi_ - c.coff), clamp = false;      // a record longer than the window
      continue;
    }
    out->span = s;
    out->status = s.status;
    out->error = s.error;
    const uint64_t np = s.next_pos;
    if (np < p.total_u()) {
      const uint64_t v = p.voff_of(np);
      out->next = Carry{v >> 16, v & 0xffff};
    } else {
      out->next = Carry{p.window_end(), np - p.total_u()};
    }
    // q_end > total_u: vend lies past this window (an indexer record that
    // straddles the window end puts np there too, and the walk goes on)
    bool ended = s.status != kOk || (s.q_end <= p.total_u() && np >= s.q_end) || (p.at_eof() && np >= p.total_u());
    if (!ended) {  // stopped at a dead position: an empty block k >= 1 starts there (finish_blocks)
      auto it = std::lower_bound(B.begin(), B.end(), np, [](const BlockInfo& b, uint64_t x) { return b.ustart < x; });
      for (; it != B.end() && it->ustart == np && !ended; ++it)
        if (it != B.begin() && it->isize == 0) ended = true;
    }
    out->ended = ended;
    return kOk;
  }
  err_ = "window planning did not converge";
  return kErrState;
}

int BamFile::all_blocks(const std::vector<BlockInfo>** out) {
  if (!have_all_blocks_) {
    all_blocks_.clear();
    uint64_t lo = 0, ubase = 0, w = window_bytes_;
    while (lo < src_.size) {
      int rc = load_window(lo, lo + w);
      if (rc != kOk) return rc;
      const auto& B = pipe_->blocks();
      if (B.empty() && !pipe_->at_eof()) {
        w *= 2;
        continue;
      }
      for (BlockInfo b : B) {
        b.ustart += ubase;
        all_blocks_.push_back(b);
      }
      ubase += pipe_->total_u();
      if (pipe_->at_eof()) break;
      lo = pipe_->window_end();
      w = window_bytes_;
    }
    have_all_blocks_ = true;
  }
  *out = &all_blocks_;
  return kOk;
}

int BamFile::read_inflated(uint64_t pos, uint64_t len, std::vector<uint8_t>* out) {
  out->clear();
  const std::vector<BlockInfo>* B = nullptr;
  int rc = all_blocks(&B);
  if (rc != kOk) return rc;
  if (len == 0 || B->empty()) return kOk;
  const BlockInfo& last = B->back();
  const uint64_t total = last.ustart + last.isize;
  if (pos >= total) return kOk;
  len = std::min(len, total - pos);
  auto first_ending_after = [&](uint64_t q) {
    return std::lower_bound(B->begin(), B->end(), q,
                            [](const BlockInfo& b, uint64_t x) { return b.ustart + b.isize <= x; });
  };
  auto a = first_ending_after(pos), e = first_ending_after(pos + len - 1);
  rc = load_window(a->coff, e->coff + e->csize);
  if (rc != kOk) return rc;
  rc = pipe_->read_stream(pos - a->ustart, len, out);
  if (rc != kOk) err_ = pipe_->error();
  return rc;
}

uint64_t BamFile::block_end_of(uint64_t pos) const {
  const auto& B = pipe_->blocks();
  const uint32_t k = pipe_->block_containing(pos);
  if (k >= B.size()) return pipe_->window_end();
  return B[k].coff + B[k].csize;
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
  put_be64(out, f.first_record_voff());  // :262-264
  // the chain starts at the header end (skipToAlignmentList :292-328) and
  // runs window by window; record ordinals continue across windows
  const uint64_t fv = f.first_record_voff();
  Carry c{fv >> 16, fv & 0xffff};
  bool cont = false;
  uint64_t ordinal = 0;
  std::vector<uint64_t> ent;
  for (;;) {
    Step st;
    int rc = f.decode_step(c, ~0ull, hbam::kIndexer, false, cont, &st);
    if (rc != kOk) return rc;
    if (st.status != kOk) {
      f.error() = st.error;
      return st.status;
    }
    rc = f.pipe().splitting_entries(st.span, (uint32_t)g, ordinal, &ent);
    if (rc != kOk) {
      f.error() = f.pipe().error();
      return rc;
    }
    for (uint64_t v : ent) put_be64(out, v);  // :273-277
    ordinal += st.span.n;
    if (st.ended) break;
    c = st.next;
    cont = true;
  }
  put_be64(out, f.file_size() << 16);  // :286
  return kOk;
}

int SplittingBAMIndexer::entries(BamFile& f, uint64_t vstart, uint64_t vend, int32_t g, uint64_t ordinal0,
                                 std::vector<uint64_t>* out, uint64_t* n_records) {
  out->clear();
  *n_records = 0;
  if (g <= 0) {
    f.error() = "Granularity must be a positive integer";
    return kErrArg;
  }
  // the indexer's chain (readAlignment / fullySkip, :340-368) over the split,
  // window by window; entries at global ordinals k*g - 1 (:273-277)
  Carry c{vstart >> 16, vstart & 0xffff};
  bool cont = false;
  uint64_t ordinal = ordinal0;
  std::vector<uint64_t> ent;
  for (;;) {
    Step st;
    int rc = f.decode_step(c, vend, hbam::kIndexer, false, cont, &st);
    if (rc != kOk) return rc;
    if (st.status != kOk) {
      f.error() = st.error;
      return st.status;
    }
    rc = f.pipe().splitting_entries(st.span, (uint32_t)g, ordinal, &ent);
    if (rc != kOk) {
      f.error() = f.pipe().error();
      return rc;
    }
    out->insert(out->end(), ent.begin(), ent.end());
    ordinal += st.span.n;
    if (st.ended) break;
    c = st.next;
    cont = true;
  }
  *n_records = ordinal - ordinal0;
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
                std::vector<uint64_t>* out, std::string* err, int32_t n_ref);

int BAMSplitGuesser::guessNextBAMRecordStarts(const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                                              std::vector<uint64_t>* out) {
  return guess_batch(f_, begs, ends, out, &f_.error(), n_ref_);
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

// ---------------------------------------------------------------------------
// BAI split calculator
// ---------------------------------------------------------------------------
int LinearBAMIndex::read(const uint8_t* d, uint64_t len, std::string* err) {
  lin_.clear();
  uint64_t p = 0;
  auto need = [&](uint64_t k) { return p + k <= len; };
  auto i32 = [&]() {
    const int32_t v = rd_i32(d + p);
    p += 4;
    return v;
  };
  if (!need(8) || memcmp(d, "BAI\1", 4) != 0) {
    *err = "Invalid file header in BAM index";
    return kErrIO;
  }
  p = 4;
  const int32_t n_ref = i32();
  if (n_ref < 0) {
    *err = "Invalid BAM index: negative reference count";
    return kErrIO;
  }
  lin_.resize((size_t)n_ref);
  for (int32_t r = 0; r < n_ref; ++r) {
    if (!need(4)) { *err = "Premature end of BAM index"; return kErrIO; }
    const int32_t n_bin = i32();
    for (int32_t b = 0; b < n_bin; ++b) {
      if (!need(8)) { *err = "Premature end of BAM index"; return kErrIO; }
      p += 4;
      const int32_t n_chunk = i32();
      if (n_chunk < 0 || !need(16ull * (uint64_t)n_chunk)) { *err = "Premature end of BAM index"; return kErrIO; }
      p += 16ull * (uint64_t)n_chunk;
    }
    if (!need(4)) { *err = "Premature end of BAM index"; return kErrIO; }
    const int32_t n_intv = i32();
    if (n_intv < 0 || !need(8ull * (uint64_t)n_intv)) { *err = "Premature end of BAM index"; return kErrIO; }
    if (n_bin > 0) {
      auto& v = lin_[(size_t)r];
      v.resize((size_t)n_intv);
      for (int32_t k = 0; k < n_intv; ++k) memcpy(&v[(size_t)k], d + p + 8ull * (uint64_t)k, 8);
    }
    p += 8ull * (uint64_t)n_intv;
  }
  return kOk;
}

// BAMInputFormat.addBAISplits (BAMInputFormat.java:322-465), for the
// FileSplits of one file in order.  Quirks kept: a contig's last linear
// entry is stepped over (`bin + 1 >= ctgBins` advances first), the last
// FileSplit is planned after the loop, and a split that no linear entry
// starts in gets a guessed start (BAMSplitGuesser, on the GPU) that also
// ends the split before it.  Where the Java code would throw a
// NullPointerException (no contig with linear entries, a guessed first
// split) this returns kErrState (unchecked in Java: getSplits does not catch
// it); a guesser I/O error is the IOException getSplits catches (:249-253).
int BAMInputFormat::addBAISplits(BamFile& f, const std::vector<FileSplit>& splits, const LinearBAMIndex& idx,
                                 std::vector<FileVirtualSplit>* out) {
  const int32_t dict = f.n_ref();
  const size_t n = splits.size();
  size_t splitsEnd = 0;
  int32_t ctgIdx = -1;
  uint32_t bin = 0;
  const std::vector<uint64_t>* linIdx = nullptr;
  size_t ctgBins = 0;
  auto npe = [&](const char* what) {
    f.error() = std::string("NullPointerException in the BAI split calculator: ") + what;
    return kErrState;
  };
  do {  // :353-357 the first contig with linear entries
    ++ctgIdx;
    linIdx = idx.getLinearIndex(ctgIdx);
    if (!linIdx) return npe("no reference sequence with a linear index");
    ctgBins = linIdx->size();
  } while (ctgBins == 0);
  uint64_t nextStart = (*linIdx)[bin], lastStart = 0;
  int64_t cur = -1;  // newSplit (index into out)
  bool lastWasGuessed = false;
  BAMSplitGuesser guesser(f);
  while (splitsEnd < n) {  // :363-445
    const FileSplit& fs = splits[splitsEnd];
    ++splitsEnd;
    if (splitsEnd >= n) break;
    const uint64_t fSplitEnd = (fs.start + fs.length) << 16;
    lastStart = nextStart;
    while (nextStart < fSplitEnd && ctgIdx < dict) {  // :380-407
      if (bin + 1 >= ctgBins) {
        do {
          ctgIdx += 1;
          bin = 0;
          if (ctgIdx >= dict) break;
          linIdx = idx.getLinearIndex(ctgIdx);
          if (!linIdx) return npe("no linear index for a dictionary sequence");
          ctgBins = linIdx->size();
        } while (ctgBins == 0);
      }
      if (ctgIdx < dict && linIdx->size() > bin) {
        nextStart = (*linIdx)[bin];
        bin++;
      }
    }
    FileVirtualSplit v;
    v.path = fs.path;
    if (fs.start == 0) {  // :409-418 from the first record
      v.vStart = f.first_record_voff();
      v.vEnd = nextStart - 1;
      out->push_back(v);
      cur = (int64_t)out->size() - 1;
    } else if (lastStart != nextStart) {  // :423-431 a linear entry starts in this split
      if (lastWasGuessed) {
        (*out)[(size_t)cur].setEndVirtualOffset(lastStart - 1);
        lastWasGuessed = false;
      }
      v.vStart = lastStart;
      v.vEnd = nextStart - 1;
      out->push_back(v);
      cur = (int64_t)out->size() - 1;
    } else {  // :432-444 guess the start
      std::vector<uint64_t> b{fs.start}, e{fs.start + fs.length}, g;
      int rc = guesser.guessNextBAMRecordStarts(b, e, &g);
      if (rc != kOk) return rc;
      const uint64_t alignedBeg = g[0];
      if (cur < 0) return npe("a guessed split with no split before it");
      (*out)[(size_t)cur].setEndVirtualOffset(alignedBeg - 1);
      lastStart = alignedBeg;
      nextStart = alignedBeg;
      v.vStart = alignedBeg;
      v.vEnd = alignedBeg + 1;
      out->push_back(v);
      cur = (int64_t)out->size() - 1;
      lastWasGuessed = true;
    }
    lastStart = nextStart;
  }
  if (splitsEnd == n && n > 0) {  // :447-459 the last split
    if (lastWasGuessed) (*out)[(size_t)cur].setEndVirtualOffset(lastStart - 1);
    const FileSplit& fs = splits[splitsEnd - 1];
    FileVirtualSplit v;
    v.path = fs.path;
    v.vStart = lastStart;
    v.vEnd = (fs.start + fs.length) << 16;
    out->push_back(v);
  }
  return kOk;
}

int BAMInputFormat::getSplits(BamFile& f, const std::vector<FileSplit>& splits, const uint8_t* sbi,
                              uint64_t sbi_len, std::vector<FileVirtualSplit>* out, const uint8_t* bai,
                              uint64_t bai_len) {
  out->clear();
  if (sbi) {
    SplittingBAMIndex idx;
    std::string err;
    if (idx.readIndex(sbi, sbi_len, &err) == kOk) {
      bool bad = false;
      int rc = addIndexedSplits(f, splits, idx, out, &bad);
      if (rc != kOk) return rc;
      if (!bad) return kOk;
      out->clear();  // "Index ... was not good. Generating probabilistic splits." (:303-306)
      return addProbabilisticSplits(f, splits, out);
    }
  }
  // no usable .splitting-bai (addIndexedSplits' IOException, :245-257): the
  // BAI split calculator when enabled and the .bai exists, else probabilistic
  if (bai) {
    LinearBAMIndex idx;
    std::string err;
    if (idx.read(bai, bai_len, &err) != kOk) {  // htsjdk's parse error is unchecked (SAMException): it propagates
      f.error() = err;
      return kErrFormat;
    }
    const int rc = addBAISplits(f, splits, idx, out);
    if (rc != kErrIO) return rc;
    out->clear();  // addBAISplits' IOException: probabilistic splits (:249-253)
  }
  return addProbabilisticSplits(f, splits, out);
}

// ---------------------------------------------------------------------------
// Host batches, the span cursor, BAMRecordReader
// ---------------------------------------------------------------------------
int HostBatch::reserve(uint64_t nn, uint64_t bytes) {
  bool ok = ref_id.resize(nn) && pos.resize(nn) && l_seq.resize(nn) && next_ref_id.resize(nn) &&
            next_pos.resize(nn) && tlen.resize(nn) && l_read_name.resize(nn) && mapq.resize(nn) && bin.resize(nn) &&
            n_cigar.resize(nn) && flag.resize(nn) && key.resize(nn) && voff.resize(nn) && rest_off.resize(nn) &&
            rest_len.resize(nn) && data.resize(bytes);
  return ok ? kOk : kErrNoMem;
}

BatchView BatchView::of(const HostBatch& h) {
  BatchView v;
  v.n = h.n;
  v.ref_id = h.ref_id.data();
  v.pos = h.pos.data();
  v.l_seq = h.l_seq.data();
  v.next_ref_id = h.next_ref_id.data();
  v.next_pos = h.next_pos.data();
  v.tlen = h.tlen.data();
  v.l_read_name = h.l_read_name.data();
  v.mapq = h.mapq.data();
  v.bin = h.bin.data();
  v.n_cigar = h.n_cigar.data();
  v.flag = h.flag.data();
  v.key = h.key.data();
  v.voff = h.voff.data();
  v.rest_off = h.rest_off.data();
  v.rest_len = h.rest_len.data();
  v.data = h.data.data();
  v.data_len = h.data_len;
  return v;
}

int fetch_span(hbam::Pipeline& p, const SpanDev& s, uint64_t k, uint64_t m, HostBatch* h, std::string* err) {
  if (m == 0) return kOk;
  const hipStream_t st = p.stream();
  const hbam::Columns& c = s.col;
  uint64_t lo = 0, last_off = 0;
  uint32_t last_len = 0;
  if (hipMemcpyAsync(&lo, s.rec_pos + k, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&last_off, c.rest_off + k + m - 1, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&last_len, c.rest_len + k + m - 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    *err = "hipMemcpy D2H failed";
    return kErrDevice;
  }
  const uint64_t hi = last_off + last_len, n0 = h->n, d0 = h->data_len;
  if (h->reserve(n0 + m, d0 + (hi - lo)) != kOk) {
    *err = "page-locked host memory for the batch";
    return kErrNoMem;
  }
  bool ok = true;
  auto cp = [&](auto& vec, const auto* src) {
    ok = ok && hipMemcpyAsync(vec.data() + n0, src + k, m * sizeof(vec[0]), hipMemcpyDeviceToHost, st) == hipSuccess;
  };
  cp(h->ref_id, c.ref_id);
  cp(h->pos, c.pos);
  cp(h->l_seq, c.l_seq);
  cp(h->next_ref_id, c.next_ref_id);
  cp(h->next_pos, c.next_pos);
  cp(h->tlen, c.tlen);
  cp(h->l_read_name, c.l_read_name);
  cp(h->mapq, c.mapq);
  cp(h->bin, c.bin);
  cp(h->n_cigar, c.n_cigar);
  cp(h->flag, c.flag);
  cp(h->key, c.key);
  cp(h->voff, c.voff);
  cp(h->rest_off, c.rest_off);
  cp(h->rest_len, c.rest_len);
  const uint8_t* src = s.data ? s.data : p.d_u();
  if (hi > lo)
    ok = ok && hipMemcpyAsync(h->data.data() + d0, src + lo, hi - lo, hipMemcpyDeviceToHost, st) == hipSuccess;
  // always drained, also after a failed enqueue: the pinned columns are freed
  // (or cached for another context) without a device-wide wait
  const bool drained = hipStreamSynchronize(st) == hipSuccess;
  if (!ok || !drained) {
    *err = "hipMemcpy D2H failed";
    return kErrDevice;
  }
  for (uint64_t i = n0; i < n0 + m; ++i) h->rest_off[i] = h->rest_off[i] - lo + d0;
  h->window_pos.push_back(lo - d0);  // window position = rest_off + this (segment base)
  h->n = n0 + m;
  h->data_len = d0 + (hi - lo);
  return kOk;
}

int BAMRecordReader::initialize(BamFile& f, const FileVirtualSplit& split) {
  // :131-133 re-entrant initialize
  f_ = &f;
  cur_span_.reset();
  b_ = BatchView();
  cur_ = 0;
  started_ = reached_end_ = have_batch_ = false;
  status_ = kOk;
  err_.clear();
  fileStart_ = split.getStartVirtualOffset() >> 16;  // :153
  virtualEnd_ = split.getEndVirtualOffset();         // :154
  next_voff_ = split.getStartVirtualOffset();
  // the iterator reads its first record in initialize (htsjdk's
  // BAMFileIndexIterator constructor advances once)
  fill();
  return status_ == kOk || b_.n > 0 ? kOk : status_;
}

bool BAMRecordReader::fill() {
  if (have_batch_ && (status_ != kOk || next_voff_ >= virtualEnd_)) return false;
  const int rc = cur_span_.next_batch(*f_, next_voff_, virtualEnd_, kBatchRecords, &b_, &next_voff_, &err_);
  have_batch_ = true;
  cur_ = 0;
  if (rc != kOk) status_ = rc;
  return b_.n > 0;
}

bool BAMRecordReader::nextKeyValue() {
  if (reached_end_) return false;
  if (started_) ++cur_;
  started_ = true;
  if (cur_ >= b_.n && !fill()) {
    reached_end_ = true;
    return false;  // status() tells a clean end from an error
  }
  view_.refID = b_.ref_id[cur_];
  view_.pos = b_.pos[cur_];
  view_.l_seq = b_.l_seq[cur_];
  view_.next_refID = b_.next_ref_id[cur_];
  view_.next_pos = b_.next_pos[cur_];
  view_.tlen = b_.tlen[cur_];
  view_.l_read_name = b_.l_read_name[cur_];
  view_.mapq = b_.mapq[cur_];
  view_.bin = b_.bin[cur_];
  view_.n_cigar = b_.n_cigar[cur_];
  view_.flag = b_.flag[cur_];
  view_.voff = b_.voff[cur_];
  view_.rest = b_.data + b_.rest_off[cur_];
  view_.rest_len = b_.rest_len[cur_];
  return true;
}

float BAMRecordReader::getProgress() const {
  if (reached_end_) return 1.0f;
  const uint64_t fileEnd = virtualEnd_ >> 16;
  if (b_.n == 0) return 0.0f;
  // before the first nextKeyValue the iterator has read record 0
  uint64_t filePos = 0;
  std::string e;
  const int rc = started_ ? cur_span_.reader_position(cur_, &filePos, &e) : cur_span_.initial_position(&filePos, &e);
  if (rc != kOk) return 0.0f;
  return (float)((double)((int64_t)filePos - (int64_t)fileStart_) / (double)(fileEnd - fileStart_ + 1));
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
