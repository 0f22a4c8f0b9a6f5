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
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "hbam_pipeline.h"

namespace hadoop_bam {

using hbam::SpanDev;

// One opened BAM (or BGZF) file: host bytes + the device pipeline + header.
class BamFile {
 public:
  static int open(const uint8_t* data, uint64_t len, int device, bool parse_header, bool check_crc,
                  std::unique_ptr<BamFile>* out, std::string* err);

  const std::vector<uint8_t>& bytes() const { return file_; }
  hbam::Pipeline& pipe() { return *pipe_; }
  uint64_t file_size() const { return file_.size(); }

  // [htsjdk] BAMFileReader.readHeader results
  int32_t n_ref() const { return n_ref_; }
  int32_t l_text() const { return (int32_t)text_.size(); }
  const std::string& text() const { return text_; }
  const std::vector<std::string>& ref_names() const { return ref_names_; }
  const std::vector<int32_t>& ref_lens() const { return ref_lens_; }
  uint64_t header_end() const { return header_end_; }
  uint64_t first_record_voff() const { return first_voff_; }

  std::string& error() { return err_; }

 private:
  int parse_header();
  std::vector<uint8_t> file_;
  std::unique_ptr<hbam::Pipeline> pipe_;
  int32_t n_ref_ = 0;
  std::string text_;
  std::vector<std::string> ref_names_;
  std::vector<int32_t> ref_lens_;
  uint64_t header_end_ = 0, first_voff_ = 0;
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
  // the indexer's read rules, entries emitted by sbi_emit.
  static int index(BamFile& f, int32_t granularity, std::vector<uint8_t>* out);
  // write-time API :175-243
  explicit SplittingBAMIndexer(int32_t granularity = DEFAULT_GRANULARITY) : granularity_(granularity) {}
  void processAlignment(uint64_t virtualOffset);  // :197-202
  void writeVirtualOffset(uint64_t virtualOffset);  // :229-232
  void finish(uint64_t inputSize);                   // :240-243
  const std::vector<uint8_t>& bytes() const { return out_; }

 private:
  int32_t granularity_;
  uint64_t count_ = 0;
  std::vector<uint8_t> out_;
};

// BAMSplitGuesser (BAMSplitGuesser.java:69-339): batched on the GPU.
class BAMSplitGuesser {
 public:
  explicit BAMSplitGuesser(BamFile& f) : f_(f) {}
  // guessNextBAMRecordStart(beg, end) for many split points; returns end when
  // nothing is found, as the reference does.
  int guessNextBAMRecordStarts(const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                               std::vector<uint64_t>* out);

 private:
  BamFile& f_;
};

// util/BGZFSplitGuesser.guessNextBGZFBlockStart(beg, end) (:64-112) for many
// split points at once (VCF/BCF BGZF inputs; BCFSplitGuesser shares the block
// search); end when nothing is found.
int guess_bgzf_batch(BamFile& f, const std::vector<uint64_t>& begs, const std::vector<uint64_t>& ends,
                     std::vector<uint64_t>* out, std::string* err);

// BAMInputFormat split planning (BAMInputFormat.java:222-318, 469-530).
class BAMInputFormat {
 public:
  // sbi: bytes of <file>.splitting-bai or nullptr (no index -> probabilistic)
  static int getSplits(BamFile& f, const std::vector<FileSplit>& splits, const uint8_t* sbi, uint64_t sbi_len,
                       std::vector<FileVirtualSplit>* out);

 private:
  static int addIndexedSplits(BamFile& f, const std::vector<FileSplit>& splits, const SplittingBAMIndex& idx,
                              std::vector<FileVirtualSplit>* out, bool* bad_index);
  static int addProbabilisticSplits(BamFile& f, const std::vector<FileSplit>& splits,
                                    std::vector<FileVirtualSplit>* out);
};

// A decoded record handed out by BAMRecordReader: the LazyBAMRecordFactory
// argument list + the variable-length block.
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

// BAMRecordReader (BAMRecordReader.java:63-233) over one FileVirtualSplit.
class BAMRecordReader {
 public:
  // static keys :81-121
  static int64_t getKey0(int32_t refIdx, int32_t alignmentStart0) {
    return (int64_t)(((uint64_t)(int64_t)refIdx << 32) | (uint64_t)(int64_t)alignmentStart0);
  }
  static int64_t getKey(int32_t refIdx, int32_t alignmentStart) { return getKey0(refIdx, alignmentStart - 1); }

  // initialize :123-184 -- decodes the whole split on the GPU
  int initialize(BamFile& f, const FileVirtualSplit& split);
  // nextKeyValue :223-232; returns false at the end or on error (see status())
  bool nextKeyValue();
  int64_t getCurrentKey() const { return h_.key[cur_]; }
  const RecordView& getCurrentValue() const { return view_; }
  float getProgress() const;  // :209-219
  int status() const { return status_; }
  const std::string& error() const { return err_; }
  void close() {}

  // bulk access (what a JNI shim hands to Java as direct ByteBuffers)
  uint64_t size() const { return n_; }
  struct Host {
    std::vector<int32_t> ref_id, pos, l_seq, next_ref_id, next_pos, tlen;
    std::vector<uint8_t> l_read_name, mapq;
    std::vector<uint16_t> bin, n_cigar, flag;
    std::vector<int64_t> key;
    std::vector<uint64_t> voff, rest_off;
    std::vector<uint32_t> rest_len;
    std::vector<uint8_t> data;  // inflated bytes of the span; rest_off is relative to data
  };
  const Host& host() const { return h_; }

 private:
  Host h_;
  uint64_t n_ = 0, cur_ = 0;
  bool started_ = false;
  int status_ = 0;
  std::string err_;
  RecordView view_{};
  uint64_t fileStart_ = 0, virtualEnd_ = 0, lastVoff_ = 0;
};

// Fetch a span decoded on the device into host vectors.
int fetch_span(hbam::Pipeline& p, const SpanDev& s, BAMRecordReader::Host* h, std::string* err);

// MurmurHash3.murmurhash3(byte[], int) (util/MurmurHash3.java:32-102) -- scalar
int64_t murmurhash3(const uint8_t* key, uint64_t len, int32_t seed);

}  // namespace hadoop_bam
