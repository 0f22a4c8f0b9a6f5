// hbam_host.h -- C++ mirror of the reference's operator interface for the BAM
// read path (org.seqdoop.hadoop_bam), sitting on the device pipeline.
//
//   FileVirtualSplit    FileVirtualSplit.java:38-126
//   SplittingBAMIndex   SplittingBAMIndex.java:41-155
//   SplittingBAMIndexer SplittingBAMIndexer.java:64-393
//   BAMSplitGuesser     BAMSplitGuesser.java:69-339 (+ BaseSplitGuesser.java:31-108)
//   BAMInputFormat      BAMInputFormat.java:205-318, 469-530
//   BAMRecordReader     BAMRecordReader.java:63-233
//
// Names, argument meaning and error behaviour follow the Java classes; Java
// exceptions become status codes (hbam.h) and the message is kept in
// BamFile::error().
//
// A BamFile reads its compressed bytes the way BAMRecordReader reads a split
// through WrapSeekable (WrapSeekable.java:42-87): only the byte ranges a
// decode touches are copied into an HBM window (or attached from a
// device-resident copy), never the whole file up front.  A span is decoded
// window by window; the next record's position is carried from one window to
// the next, so device memory is bounded by the window size whatever the file
// size.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "hbam_pipeline.h"

namespace hadoop_bam {

using hbam::SpanDev;

constexpr uint64_t kDefaultWindowBytes = 4ull << 30;  // hadoopbam.gpu.window-bytes default
constexpr uint64_t kDropinWindowBytes = 256ull << 20;  // hbam_decode_span windows when the property is unset

// Page-locked host array (batch columns handed to a JNI caller as direct
// ByteBuffers; D2H copies into it run at the PCIe rate).
template <typename T>
class PinnedVec {
 public:
  PinnedVec() = default;
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  ~PinnedVec() { release(); }
  bool resize(size_t n);  // keeps the first min(n, size()) elements
  size_t size() const { return n_; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  void release();

 private:
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

// Where a BamFile's compressed bytes come from.
struct Source {
  hbam::HostSource host;          // the file's host bytes (copy, pread of the path, reader callback); invalid: device only
  uint64_t size = 0;              // file length
  std::vector<uint8_t> owned;     // hbam_open_mem copy
  int fd = -1;                    // hbam_open: the path (mapped; its length checked before each read)
  void* map = nullptr;            // hbam_open: read-only mmap of the path
  size_t map_len = 0;
  hbam::DevBuf<uint8_t> dev;      // device-resident bytes [dev_lo, dev_hi) (+ kFilePad zeros)
  uint64_t dev_lo = 0, dev_hi = 0;
  uint64_t bytes_read = 0;        // host -> HBM bytes copied so far (window loads + prefetch)
  ~Source();
};

// Where a span continues: the block at file offset coff, stream offset upos
// from its start (a voff when upos <= 0xffff; the indexer's skip of a record
// longer than a window may carry further).
struct Carry {
  uint64_t coff = 0, upos = 0;
  uint64_t voff() const { return (coff << 16) | (upos & 0xffff); }
};

// One window's part of a span.
struct Step {
  SpanDev span;             // records of this window (device)
  Carry next;               // where the span continues
  bool ended = true;        // span exhausted (span end, end of stream, error)
  int status = 0;           // status of the record that ended the span early
  std::string error;
};

struct OpenOptions {
  int device = 0;
  bool parse_header = true;
  bool check_crc = false;
  int stringency = hbam::kStrict;
  uint64_t window_bytes = kDefaultWindowBytes;
  bool parallel_reads = false;  // a reader callback may run on several threads at once
  uint64_t batch_records = 0;   // hbam_decode_span's max_records, when the caller knows it
};

// One opened BAM (or BGZF) file on one GPU.
class BamFile {
 public:
  // whole-file sources: an in-memory copy, an mmap of a path, or a device
  // copy of host bytes (hbam_gpu: the file resident in HBM)
  static int open_memory(const uint8_t* data, uint64_t len, const OpenOptions& o, std::unique_ptr<BamFile>* out,
                         std::string* err);
  static int open_path(const char* path, const OpenOptions& o, std::unique_ptr<BamFile>* out, std::string* err);
  // a file of `size` bytes read through a positioned-read callback
  // (hbam_open_reader: a Hadoop FSDataInputStream through JNI)
  static int open_reader(uint64_t size, hbam::HostSource::ReadFn fn, void* user, const OpenOptions& o,
                         std::unique_ptr<BamFile>* out, std::string* err);
  static int open_device_copy(const uint8_t* data, uint64_t len, const OpenOptions& o, std::unique_ptr<BamFile>* out,
                              std::string* err);

  ~BamFile() { src_.dev.release(); }  // before pipe_, whose streams own it
  hbam::Pipeline& pipe() { return *pipe_; }
  uint64_t file_size() const { return src_.size; }
  uint64_t bytes_read() const { return src_.bytes_read; }
  uint64_t window_bytes() const { return window_bytes_; }
  bool window_explicit() const { return window_explicit_; }
  // file bytes [lo, hi) already in HBM (prefetch, or a device copy)
  bool resident(uint64_t lo, uint64_t hi) const { return src_.dev.p && lo >= src_.dev_lo && hi <= src_.dev_hi; }
  void set_window_bytes(uint64_t w) { window_bytes_ = w < (1ull << 16) ? (1ull << 16) : w; }

  // [htsjdk] BAMFileReader.readHeader results
  int32_t n_ref() const { return n_ref_; }
  int32_t l_text() const { return (int32_t)text_.size(); }
  const std::string& text() const { return text_; }
  const std::vector<std::string>& ref_names() const { return ref_names_; }
  const std::vector<int32_t>& ref_lens() const { return ref_lens_; }
  uint64_t first_record_voff() const { return first_voff_; }

  std::string& error() { return err_; }

  // Copy file bytes [lo, hi) into HBM now; windows inside the range then
  // attach to it instead of reading the host (bench: inputs resident in HBM).
  int prefetch(uint64_t lo, uint64_t hi);
  // the next load re-attaches / re-copies and re-locates (timed passes)
  void invalidate_window() { win_lo_ = ~0ull; }
  // Load the window [lo, hi) (clipped to the file) and locate its blocks.
  int load_window(uint64_t lo, uint64_t hi, bool free_start = false, bool host_only = false);

  // Decode the part of FileVirtualSplit [.., vend) that starts at `from`
  // and lies in one window.  continuation: `from` is the carry of the
  // previous step (not a reader seek).
  // window: compressed bytes per window (0 = window_bytes()); next_window:
  // the size of the caller's next window, staged while this one decodes
  // (0 = window)
  int decode_step(Carry from, uint64_t vend, hbam::ChainMode mode, bool decode, bool continuation,
                  Step* out, uint64_t window = 0, uint64_t next_window = 0);
  // window of the drop-in batch path (hbam_decode_span): hadoopbam.gpu.window-bytes
  // when set, else kDropinWindowBytes -- several windows per split, so that
  // one window's batches cross PCIe while the next decodes
  uint64_t dropin_window_bytes() const {
    return window_explicit_ ? window_bytes_ : std::min(window_bytes_, kDropinWindowBytes);
  }

  // Every BGZF block of the file (window by window; cached).  ustart is the
  // offset in the whole inflated stream.
  int all_blocks(const std::vector<hbam::BlockInfo>** out);
  // Inflated bytes [pos, pos + len) of the whole stream.
  int read_inflated(uint64_t pos, uint64_t len, std::vector<uint8_t>* out);
  // file offset just past the block holding window position `pos` (window of the last step)
  uint64_t block_end_of(uint64_t pos) const;

 private:
  BamFile() = default;
  int init(const OpenOptions& o, std::string* err);
  int parse_header();
  Source src_;
  std::unique_ptr<hbam::Pipeline> pipe_;
  uint64_t win_lo_ = ~0ull, win_hi_ = 0;  // the loaded window
  uint64_t staged_lo_ = 0, staged_hi_ = 0;  // the range handed to Pipeline::stage last
  bool win_free_ = false;
  uint64_t window_bytes_ = kDefaultWindowBytes;
  bool window_explicit_ = false;
  int32_t n_ref_ = 0;
  std::string text_;
  std::vector<std::string> ref_names_;
  std::vector<int32_t> ref_lens_;
  uint64_t first_voff_ = 0;
  std::vector<hbam::BlockInfo> all_blocks_;
  bool have_all_blocks_ = false;
  std::string err_;
};

// FileVirtualSplit (FileVirtualSplit.java:38-126): vStart inclusive, vEnd exclusive.
struct FileVirtualSplit {
  std::string path;
  uint64_t vStart = 0, vEnd = 0;
  uint64_t getStartVirtualOffset() const { return vStart; }
  uint64_t getEndVirtualOffset() const { return vEnd; }
  void setEndVirtualOffset(uint64_t v) { vEnd = v; }
  // :73-78 inexact length
  uint64_t getLength() const {
    const uint64_t hs = vStart & ~0xffffull, he = vEnd & ~0xffffull;
    return he == hs ? ((vEnd & 0xffff) - (vStart & 0xffff)) : he - hs;
  }
};

// Hadoop FileSplit (byte range) -- input of getSplits.
struct FileSplit {
  std::string path;
  uint64_t start = 0, length = 0;
};

// SplittingBAMIndex (SplittingBAMIndex.java:41-155).
class SplittingBAMIndex {
 public:
  // readIndex :52-72 (IOException -> HBAM_E_IO)
  int readIndex(const uint8_t* data, uint64_t len, std::string* err);
  // :78-83 floor / strictly-higher lookups; false = Java null
  bool prevAlignment(uint64_t filePos, uint64_t* out) const;
  bool nextAlignment(uint64_t filePos, uint64_t* out) const;
  size_t size() const { return offsets_.size(); }
  uint64_t bamSize() const { return offsets_.empty() ? 0 : (*offsets_.rbegin()) >> 16; }
  std::vector<uint64_t> getVirtualOffsets() const { return {offsets_.begin(), offsets_.end()}; }

 private:
  std::set<uint64_t> offsets_;
};

// SplittingBAMIndexer (SplittingBAMIndexer.java:64-393).
class SplittingBAMIndexer {
 public:
  static constexpr int DEFAULT_GRANULARITY = 4096;  // :70
  // index(in, out, inputSize, granularity) :248-290 -- GPU record chain under
  // the indexer's read rules, window by window, entries by global ordinal.
  static int index(BamFile& f, int32_t granularity, std::vector<uint8_t>* out);
  // the part of index() one split contributes (multi-GPU):
  // entries of the records of [vstart, vend), the first having global ordinal
  // ordinal0; *n_records = records of the split
  static int entries(BamFile& f, uint64_t vstart, uint64_t vend, int32_t granularity, uint64_t ordinal0,
                     std::vector<uint64_t>* out, uint64_t* n_records);
  // write-time API :175-243 (BAMRecordWriter.java:145-149 drives it): the
  // entries of a run of record voffs, computed on the GPU (k_sbi_emit)
  explicit SplittingBAMIndexer(int32_t granularity = DEFAULT_GRANULARITY) : granularity_(granularity) {}
  void processAlignment(uint64_t virtualOffset);    // :197-202
  void writeVirtualOffset(uint64_t virtualOffset);  // :229-232
  void finish(uint64_t inputSize);                  // :240-243
  const std::vector<uint8_t>& bytes() const { return out_; }

 private:
  int32_t granularity_;
  uint64_t count_ = 0;
  std::vector<uint8_t> out_;
};

// BAMSplitGuesser (BAMSplitGuesser.java:69-339): batched on the GPU over
// windows around the split points.
class BAMSplitGuesser {
 public:
  explicit BAMSplitGuesser(BamFile& f) : f_(f) {}
  // BAMSplitGuesser(SeekableStream, InputStream headerStream, Configuration)
  // (BAMSplitGuesser.java:93-103): the reference count of a header read from
  // another stream than the data's (< 0: the data file's own header)
  BAMSplitGuesser(BamFile& f, int32_t header_n_ref) : f_(f), n_ref_(header_n_ref) {}
  // guessNextBAMRecordStart(beg, end) for many split points; returns end when
  // nothing is found, as the reference does.
  int guessNextBAMRecordStarts(const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                               std::vector<uint64_t>* out);

 private:
  BamFile& f_;
  int32_t n_ref_ = -1;
};

// util/BGZFSplitGuesser.guessNextBGZFBlockStart(beg, end) (:64-112) for many
// split points at once (VCF/BCF BGZF inputs; BCFSplitGuesser shares the block
// search); end when nothing is found.
int guess_bgzf_batch(BamFile& f, const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                     std::vector<uint64_t>* out, std::string* err);

// BAMInputFormat split planning (BAMInputFormat.java:222-318, 469-530).
// The linear index of a .bai (SAM spec 5.2; htsjdk CachingBAMFileIndex as
// LinearBAMIndex reads it, src/main/java/htsjdk/samtools/LinearBAMIndex.java):
// per reference its 16 kbp-window virtual offsets; a reference with no bins
// has none.
class LinearBAMIndex {
 public:
  int read(const uint8_t* d, uint64_t len, std::string* err);
  // nullptr past the last reference (htsjdk's query returns null there)
  const std::vector<uint64_t>* getLinearIndex(int32_t ctg) const {
    return ctg >= 0 && (size_t)ctg < lin_.size() ? &lin_[(size_t)ctg] : nullptr;
  }

 private:
  std::vector<std::vector<uint64_t>> lin_;
};

class BAMInputFormat {
 public:
  // sbi: bytes of <file>.splitting-bai or nullptr (no index -> probabilistic);
  // bai: bytes of the file's .bai or nullptr -- with the BAI split calculator
  // enabled (hadoopbam.bam.enable-bai-splitter) it plans when the
  // .splitting-bai is absent or bad (BAMInputFormat.java:241-257)
  static int getSplits(BamFile& f, const std::vector<FileSplit>& splits, const uint8_t* sbi, uint64_t sbi_len,
                       std::vector<FileVirtualSplit>* out, const uint8_t* bai = nullptr, uint64_t bai_len = 0);

 private:
  static int addBAISplits(BamFile& f, const std::vector<FileSplit>& splits, const LinearBAMIndex& idx,
                          std::vector<FileVirtualSplit>* out);
  static int addIndexedSplits(BamFile& f, const std::vector<FileSplit>& splits, const SplittingBAMIndex& idx,
                              std::vector<FileVirtualSplit>* out, bool* bad_index);
  static int addProbabilisticSplits(BamFile& f, const std::vector<FileSplit>& splits,
                                    std::vector<FileVirtualSplit>* out);
};

// Host copy of a run of decoded records: the LazyBAMRecordFactory argument
// list + key + voff + the variable-length block of each record (owning;
// hbam_decode_writables and whole-split batches).
struct HostBatch {
  PinnedVec<int32_t> ref_id, pos, l_seq, next_ref_id, next_pos, tlen;
  PinnedVec<uint8_t> l_read_name, mapq;
  PinnedVec<uint16_t> bin, n_cigar, flag;
  PinnedVec<int64_t> key;
  PinnedVec<uint64_t> voff, rest_off;
  PinnedVec<uint32_t> rest_len;
  PinnedVec<uint8_t> data;  // inflated bytes of the records; rest_off is relative to data
  uint64_t n = 0, data_len = 0;
  std::vector<uint64_t> window_pos;  // window position of data[0] per window segment (progress)
  int reserve(uint64_t n, uint64_t bytes);
};

// The host columns of one batch as handed to the caller (the hbam_batch
// field set): pointers into a HostBatch or into a page-locked batch slot.
struct BatchView {
  uint64_t n = 0;
  const int32_t *ref_id = nullptr, *pos = nullptr, *l_seq = nullptr, *next_ref_id = nullptr, *next_pos = nullptr,
                *tlen = nullptr;
  const uint8_t *l_read_name = nullptr, *mapq = nullptr;
  const uint16_t *bin = nullptr, *n_cigar = nullptr, *flag = nullptr;
  const int64_t* key = nullptr;
  const uint64_t *voff = nullptr, *rest_off = nullptr;
  const uint32_t* rest_len = nullptr;
  const uint8_t* data = nullptr;  // rest_off is relative to data
  uint64_t data_len = 0;
  static BatchView of(const HostBatch& h);
};

// Records [k, k + m) of a device span appended to h at record h->n (columns
// and their bytes; D2H on the pipeline stream into page-locked memory).
int fetch_span(hbam::Pipeline& p, const SpanDev& s, uint64_t k, uint64_t m, HostBatch* h, std::string* err);

// A split being read in bounded batches (BAMRecordReader's iterator,
// hbam_decode_span).  The split is decoded window by window
// (BamFile::dropin_window_bytes) and each decoded window's records are
// exported from the pipeline into one of two device slots, so that:
//   * while the caller holds batch j, batch j+1 is already crossing PCIe
//     (SDMA copies of its column slices and bytes; two page-locked host
//     slots in turn);
//   * when a window's first batch is handed out, the next window is decoded
//     (its compressed bytes go host->HBM while this window's batches go
//     HBM->host: the link is full duplex with the copy engines).
// A batch holds records of one window.  max_records = 0 returns the rest of
// the split in one owning HostBatch (several windows appended).
class SpanCursor {
 public:
  // window id of a split read from the host: 32 MiB, doubling up to `full`
  // (HBAM_DROPIN_RAMP="first MiB,growth"), so decoding starts after a small copy
  static uint64_t ramp_window(uint64_t full, uint64_t id);
  SpanCursor() = default;
  SpanCursor(const SpanCursor&) = delete;
  SpanCursor& operator=(const SpanCursor&) = delete;
  ~SpanCursor();
  // Up to max_records records (0 = the rest of the split) starting at vstart;
  // *next_voff = where the next call continues (>= vend when the split is
  // exhausted).  A vstart equal to the previous call's *next_voff continues
  // the same split without re-decoding.  *out stays valid until the next call.
  int next_batch(BamFile& f, uint64_t vstart, uint64_t vend, uint64_t max_records, BatchView* out,
                 uint64_t* next_voff, std::string* err);
  // pin both batch slots for batches of m records on a helper thread (device:
  // the ctx's device, before the first batch has set it)
  void start_prealloc(uint64_t m, int device = -1);
  // device view of the records of the last batch when they lie in one window
  bool last_batch_span(SpanDev* out) const;
  // BAMRecordReader.getProgress's in.position() after record i of the last
  // batch (htsjdk's iterator has read the record after it)
  int reader_position(uint64_t i, uint64_t* pos, std::string* err) const;
  // ... before the first record is returned (htsjdk has read record 0)
  int initial_position(uint64_t* pos, std::string* err) const;
  bool valid() const { return valid_; }
  // forget the split (waits for this cursor's copies in flight)
  void reset();

 private:
  struct Window {  // one decoded window's records, exported out of the pipeline
    hbam::DevBuf<uint8_t> cols, bytes;
    hbam::DevBuf<uint8_t> packed;  // the columns again, batch-major in batches of pack_m (one D2H per batch)
    hbam::DevBuf<uint8_t> rests;   // the records' rests back to back (k_pack_rests): what a batch sends
    uint64_t pack_m = 0;
    hbam::Columns col{};
    uint64_t* rec_pos = nullptr;  // n + 1 entries: slot byte offsets, [n] = nbytes
    uint64_t n = 0, nbytes = 0, base_pos = 0, id = 0;
    std::shared_ptr<const std::vector<hbam::BlockInfo>> blocks;  // block table (positions)
    Carry next;
    bool ended = true;
    int status = 0;
    std::string error;
    hipEvent_t ready = nullptr;  // export done
  };
  struct Slot {  // a page-locked batch: ColLayout(m) columns, then the records' rests
    uint8_t* mem = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool busy = false;            // copies queued
    bool packed = false;          // columns came batch-major (rest_off already batch-relative)
    uint64_t win = 0, k = 0, m = 0, start = 0, end = 0, ahead_end = 0, next_voff = 0;
  };
  int ensure_streams(hbam::Pipeline& p, std::string* err);
  int decode_window(BamFile& f, Carry from, bool cont, uint64_t m, Window* w, std::string* err);
  int issue(const Window& w, uint64_t k, uint64_t m, Slot* s, std::string* err);
  // m capped so that the batch's rest bytes fit a Java direct buffer (an int
  // capacity and int positions: GpuBAMRecordReader.recordAt): the largest
  // m' <= m whose rests [k, k + m') take at most batch_data_cap() bytes
  // (at least one record)
  int capped(const Window& w, uint64_t k, uint64_t m, uint64_t* out, std::string* err);
  int drain();
  int next_batch_all(BamFile& f, uint64_t vstart, uint64_t vend, BatchView* out, uint64_t* next_voff,
                     std::string* err);
  uint64_t block_end(const std::vector<hbam::BlockInfo>& B, uint64_t pos) const;

  bool valid_ = false;
  uint64_t vend_ = 0, next_voff_ = 0;
  hipStream_t d2h_ = nullptr, meta_ = nullptr;
  int device_ = -1;
  hbam::StreamSet own_;            // the pipeline stream + d2h_ + meta_
  // owner of the window slots' device buffers: the pipeline stream only (the
  // export writes them there).  A slot is decoded into again only after every
  // batch of its previous window has landed, so its regrowth need not wait for
  // the batch copies of the other slot's window in flight on d2h_.
  hbam::StreamSet slot_owner_;
  Window win_[2];
  uint64_t front_ = 0, nwin_ = 0;  // window ids: front_ = the one being handed out; nwin_ decoded so far
  uint64_t k_ = 0;                 // next record of the front window
  Slot slot_[2];
  // the first batches' page-locked slots, mapped and pinned on a helper
  // thread while the first window decodes (joined before a slot is used)
  std::thread prealloc_;
  void join_prealloc();
  int cur_ = -1;                   // slot of the last batch handed out
  uint64_t* small_ = nullptr;      // page-locked scratch for the boundary reads
  // the last batch: where its records came from (positions / encode)
  uint64_t last_win_ = 0, last_k_ = 0, last_m_ = 0, last_start_ = 0, last_ahead_end_ = 0, last_base_pos_ = 0;
  bool last_bounded_ = false;
  BatchView last_view_;
  std::shared_ptr<const std::vector<hbam::BlockInfo>> last_blocks_;
  // max_records = 0: the whole rest of the split, appended window by window
  HostBatch all_;
  std::vector<std::pair<uint64_t, std::shared_ptr<const std::vector<hbam::BlockInfo>>>> all_seg_;  // first record, blocks
  Step all_step_;
  bool all_one_window_ = false;
};

// BAMRecordReader (BAMRecordReader.java:63-233) over one FileVirtualSplit.
class BAMRecordReader {
 public:
  static constexpr uint64_t kBatchRecords = 1 << 20;  // records per device->host batch
  // static keys :81-121
  static int64_t getKey0(int32_t refIdx, int32_t alignmentStart0) {
    return (int64_t)(((uint64_t)(int64_t)refIdx << 32) | (uint64_t)(int64_t)alignmentStart0);
  }
  static int64_t getKey(int32_t refIdx, int32_t alignmentStart) { return getKey0(refIdx, alignmentStart - 1); }

  // initialize :123-184 -- positions the cursor at the split start; records
  // are decoded on the GPU in batches as nextKeyValue reaches them
  int initialize(BamFile& f, const FileVirtualSplit& split);
  // nextKeyValue :223-232; returns false at the end or on error (see status())
  bool nextKeyValue();
  int64_t getCurrentKey() const { return b_.key[cur_]; }
  struct RecordView {
    int32_t refID, pos, l_seq, next_refID, next_pos, tlen;
    uint8_t l_read_name, mapq;
    uint16_t bin, n_cigar, flag;
    uint64_t voff;
    const uint8_t* rest;
    uint32_t rest_len;
    int32_t getAlignmentStart() const { return pos + 1; }
    int32_t getMateAlignmentStart() const { return next_pos + 1; }
  };
  const RecordView& getCurrentValue() const { return view_; }
  float getProgress() const;  // :209-219
  int status() const { return status_; }
  const std::string& error() const { return err_; }
  void close() {}

 private:
  bool fill();
  BamFile* f_ = nullptr;
  SpanCursor cur_span_;
  BatchView b_;
  uint64_t cur_ = 0, next_voff_ = 0;
  bool started_ = false, reached_end_ = false, have_batch_ = false;
  int status_ = 0;
  std::string err_;
  RecordView view_{};
  uint64_t fileStart_ = 0, virtualEnd_ = 0;
};

// MurmurHash3.murmurhash3(byte[], int) (util/MurmurHash3.java:32-102) -- scalar
int64_t murmurhash3(const uint8_t* key, uint64_t len, int32_t seed);

}  // namespace hadoop_bam
