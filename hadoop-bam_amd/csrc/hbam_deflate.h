// hbam_deflate.h -- raw DEFLATE of one BGZF block payload, restating zlib
// 1.2.11's deflate_fast / deflate_slow / trees.c (levels 1-9; zlib is what
// java.util.zip.Deflater wraps) so that the output is byte-identical to
// [htsjdk] BlockCompressedOutputStream.deflateBlock: one Deflater(level,
// nowrap=true), reset() per block, setInput + finish + deflate(buf, 0, 65518).
//
// The whole payload is in the window after the first fill_window (payload
// <= 65536 = window_size), so the window is a view over the input.  The
// single slide of a payload >= wsize + MAX_DIST copies [wsize, len) down
// (1.2.11: wsize - more bytes), applied by the view as an index remap.
// Window bytes past the payload end (zeroed by zlib's high_water logic on a
// fresh stream, stale data of earlier blocks on a reset() one) are read by
// longest_match but never decide a match: nice_match is capped at lookahead
// and a longer capped match loses to prev_length.  deflate_check runs both
// Deflater lifecycles against zlib to hold that.
//
// One call = one block; state lives in a caller-provided arena (global
// memory on the GPU, one arena per lane; host memory in the CPU check).
// Everything here is __host__ __device__ so the same code is checked
// against system zlib on the host (tools/deflate_check.cpp) and runs in
// k_deflate_blocks (hbam_deflate.hip).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define DFL_HD __host__ __device__
#define DFL_NOINLINE __attribute__((noinline))
#else
#define DFL_HD
#define DFL_NOINLINE
#endif

namespace hbam {
namespace dfl {

constexpr int kWSize = 32768;            // w_size (windowBits 15)
constexpr int kWMask = kWSize - 1;
constexpr int kMinMatch = 3, kMaxMatch = 258;
constexpr int kMinLookahead = kMaxMatch + kMinMatch + 1;  // 262
constexpr int kMaxDist = kWSize - kMinLookahead;          // 32506
constexpr int kHashSize = 32768, kHashMask = kHashSize - 1, kHashShift = 5;  // memLevel 8
constexpr int kLitBufSize = 16384;       // 1 << (memLevel + 6)
constexpr int kTooFar = 4096;
constexpr int kLCodes = 286, kDCodes = 30, kBlCodes = 19, kLiterals = 256, kEndBlock = 256;
constexpr int kHeapSize = 2 * kLCodes + 1;  // 573
constexpr int kMaxBits = 15, kMaxBlBits = 7;
constexpr uint32_t kOutCap = 65536 - 18;  // htsjdk compressedBuffer (MAX_COMPRESSED_BLOCK_SIZE - header)

struct Config {
  uint16_t good, lazy, nice, chain;
};
// deflate.c configuration_table: levels 1..3 run deflate_fast, 4..9 deflate_slow
DFL_HD inline Config level_config(int level) {
  switch (level) {
    case 1: return {4, 4, 8, 4};
    case 2: return {4, 5, 16, 8};
    case 3: return {4, 6, 32, 32};
    case 4: return {4, 4, 16, 16};
    case 5: return {8, 16, 32, 32};
    case 6: return {8, 16, 128, 128};
    case 7: return {8, 32, 128, 256};
    case 8: return {32, 128, 258, 1024};
    default: return {32, 258, 258, 4096};
  }
}

// trees.c static tables (tr_static_init), built once on the host.
struct Tables {
  uint16_t sl_code[288];
  uint8_t sl_len[288];
  uint16_t sd_code[30];
  uint8_t sd_len[30];
  uint8_t length_code[256];
  uint8_t dist_code[512];
  int32_t base_length[29];
  int32_t base_dist[30];
};

DFL_HD inline int extra_lbits(int c) {
  return (c < 8 || c == 28) ? 0 : (c - 4) >> 2;
}
DFL_HD inline int extra_dbits(int c) { return c < 4 ? 0 : (c - 2) >> 1; }
DFL_HD inline int extra_blbits(int c) { return c == 16 ? 2 : c == 17 ? 3 : c == 18 ? 7 : 0; }
DFL_HD inline int bl_order(int i) {
  const uint8_t o[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  return o[i];
}
DFL_HD inline unsigned bi_reverse(unsigned code, int len) {
  unsigned res = 0;
  do {
    res |= code & 1;
    code >>= 1, res <<= 1;
  } while (--len > 0);
  return res >> 1;
}

// gen_codes (trees.c): canonical codes from bit lengths
DFL_HD inline void gen_codes(uint16_t* code_out, const uint8_t* lens, int max_code, const uint16_t* bl_count) {
  uint16_t next_code[kMaxBits + 1];
  unsigned code = 0;
  for (int bits = 1; bits <= kMaxBits; bits++) {
    code = (code + bl_count[bits - 1]) << 1;
    next_code[bits] = (uint16_t)code;
  }
  for (int n = 0; n <= max_code; n++) {
    int len = lens[n];
    if (len == 0) continue;
    code_out[n] = (uint16_t)bi_reverse(next_code[len]++, len);
  }
}

inline void build_tables(Tables* t) {
  int length = 0, code;
  for (code = 0; code < 28; code++) {
    t->base_length[code] = length;
    for (int n = 0; n < (1 << extra_lbits(code)); n++) t->length_code[length++] = (uint8_t)code;
  }
  t->base_length[28] = 0;
  t->length_code[length - 1] = (uint8_t)code;
  int dist = 0;
  for (code = 0; code < 16; code++) {
    t->base_dist[code] = dist;
    for (int n = 0; n < (1 << extra_dbits(code)); n++) t->dist_code[dist++] = (uint8_t)code;
  }
  dist >>= 7;
  for (; code < kDCodes; code++) {
    t->base_dist[code] = dist << 7;
    for (int n = 0; n < (1 << (extra_dbits(code) - 7)); n++) t->dist_code[256 + dist++] = (uint8_t)code;
  }
  uint16_t bl_count[kMaxBits + 1] = {0};
  int n = 0;
  while (n <= 143) t->sl_len[n++] = 8, bl_count[8]++;
  while (n <= 255) t->sl_len[n++] = 9, bl_count[9]++;
  while (n <= 279) t->sl_len[n++] = 7, bl_count[7]++;
  while (n <= 287) t->sl_len[n++] = 8, bl_count[8]++;
  for (int i = 0; i < 288; ++i) t->sl_code[i] = 0;
  gen_codes(t->sl_code, t->sl_len, 287, bl_count);
  for (n = 0; n < kDCodes; n++) t->sd_code[n] = (uint16_t)bi_reverse((unsigned)n, 5), t->sd_len[n] = 5;
}

// Per-block working state (one arena per concurrent block).
struct alignas(16) Arena {
  uint16_t head[kHashSize];
  uint16_t prev[kWSize];
  uint16_t d_buf[kLitBufSize];
  uint8_t l_buf[kLitBufSize];
  // ct_data of the three trees: fc = Freq|Code, dl = Dad|Len (zlib unions)
  uint16_t lfc[kHeapSize], ldl[kHeapSize];
  uint16_t dfc[2 * kDCodes + 1], ddl[2 * kDCodes + 1];
  uint16_t bfc[2 * kBlCodes + 1], bdl[2 * kBlCodes + 1];
  uint16_t heap[kHeapSize];
  uint8_t depth[kHeapSize];
  uint16_t bl_count[kMaxBits + 1];
};

struct Tree {  // tree_desc
  uint16_t* fc;
  uint16_t* dl;
  const uint8_t* slen;  // static tree lengths (nullptr for bl)
  int kind;             // 0 lit/len, 1 dist, 2 bit lengths
  int elems, max_length, base;
  int max_code;
};

DFL_HD inline int tree_extra(int kind, int i) {
  return kind == 0 ? extra_lbits(i) : kind == 1 ? extra_dbits(i) : extra_blbits(i);
}

struct Out {  // pending output (send_bits / put_byte over a bounded buffer)
  uint8_t* buf;
  uint32_t cap, n;
  uint64_t bb;  // bit buffer, LSB first
  int nb;
  bool overflow;
  DFL_HD void byte(uint8_t b) {
    if (n < cap)
      buf[n] = b;
    else
      overflow = true;
    n++;
  }
  DFL_HD void bits(unsigned v, int len) {
    bb |= (uint64_t)v << nb;
    nb += len;
    while (nb >= 8) {
      byte((uint8_t)bb);
      bb >>= 8;
      nb -= 8;
    }
  }
  DFL_HD void windup() {  // bi_windup
    if (nb > 0) byte((uint8_t)bb);
    bb = 0;
    nb = 0;
  }
};

// the emulated zlib window: a view over the payload
struct Win {
  const uint8_t* in;
  uint32_t len;
  uint32_t copied;  // bytes moved down by the slide (len - wsize)
  bool slid;
  DFL_HD uint8_t pre(uint32_t y) const { return y < len ? in[y] : 0; }
  DFL_HD uint8_t win(uint32_t x) const {
    if (slid && x < copied) return pre(x + kWSize);
    return pre(x);
  }
};

// state touched only when a block is flushed (trees, bit writer): kept apart
// from the hot matching state so the out-of-line flush_block does not force
// the match loop's variables into scratch memory
struct Cold {
  Arena* a;
  const Tables* t;
  Win w;
  uint32_t last_lit;
  uint32_t opt_len, static_len;
  Tree l, d, b;
  Out out;
  DFL_HD uint8_t win(uint32_t x) const { return w.win(x); }
};

struct State {
  Win w;
  Arena* a;
  const Tables* t;
  Config cfg;
  uint32_t strstart, lookahead;
  int32_t block_start;
  uint32_t match_start, prev_match, match_length, prev_length;
  int match_available;
  uint32_t ins_h;
  uint32_t last_lit;
  Cold* c;
  DFL_HD uint8_t win(uint32_t x) const { return w.win(x); }
};

DFL_HD inline void insert_string(State& s, uint32_t str, uint32_t* match_head) {
  s.ins_h = ((s.ins_h << kHashShift) ^ s.win(str + kMinMatch - 1)) & kHashMask;
  *match_head = s.a->prev[str & kWMask] = s.a->head[s.ins_h];
  s.a->head[s.ins_h] = (uint16_t)str;
}

DFL_HD inline void init_block(Cold& s) {
  for (int n = 0; n < kLCodes; n++) s.l.fc[n] = 0;
  for (int n = 0; n < kDCodes; n++) s.d.fc[n] = 0;
  for (int n = 0; n < kBlCodes; n++) s.b.fc[n] = 0;
  s.l.fc[kEndBlock] = 1;
  s.opt_len = s.static_len = 0;
  s.last_lit = 0;
}

DFL_HD inline bool smaller(const uint16_t* fc, const uint8_t* depth, int n, int m) {
  return fc[n] < fc[m] || (fc[n] == fc[m] && depth[n] <= depth[m]);
}

DFL_HD inline void pqdownheap(Cold& s, const uint16_t* fc, int k, int heap_len) {
  uint16_t* heap = s.a->heap;
  const uint8_t* depth = s.a->depth;
  int v = heap[k];
  int j = k << 1;
  while (j <= heap_len) {
    if (j < heap_len && smaller(fc, depth, heap[j + 1], heap[j])) j++;
    if (smaller(fc, depth, v, heap[j])) break;
    heap[k] = heap[j];
    k = j;
    j <<= 1;
  }
  heap[k] = (uint16_t)v;
}

DFL_HD inline void gen_bitlen(Cold& s, Tree& tr, int heap_max) {
  uint16_t* fc = tr.fc;
  uint16_t* dl = tr.dl;
  uint16_t* bl_count = s.a->bl_count;
  uint16_t* heap = s.a->heap;
  const int max_code = tr.max_code, max_length = tr.max_length, base = tr.base;
  int overflow = 0;
  for (int bits = 0; bits <= kMaxBits; bits++) bl_count[bits] = 0;
  dl[heap[heap_max]] = 0;  // root
  int h;
  for (h = heap_max + 1; h < kHeapSize; h++) {
    int n = heap[h];
    int bits = dl[dl[n]] + 1;
    if (bits > max_length) bits = max_length, overflow++;
    dl[n] = (uint16_t)bits;
    if (n > max_code) continue;
    bl_count[bits]++;
    int xbits = 0;
    if (n >= base) xbits = tree_extra(tr.kind, n - base);
    unsigned f = fc[n];
    s.opt_len += f * (unsigned)(bits + xbits);
    if (tr.slen) s.static_len += f * (unsigned)(tr.slen[n] + xbits);
  }
  if (overflow == 0) return;
  do {
    int bits = max_length - 1;
    while (bl_count[bits] == 0) bits--;
    bl_count[bits]--;
    bl_count[bits + 1] += 2;
    bl_count[max_length]--;
    overflow -= 2;
  } while (overflow > 0);
  for (int bits = max_length; bits != 0; bits--) {
    int n = bl_count[bits];
    while (n != 0) {
      int m = heap[--h];
      if (m > max_code) continue;
      if ((unsigned)dl[m] != (unsigned)bits) {
        s.opt_len += (uint32_t)(((long)bits - (long)dl[m]) * (long)fc[m]);
        dl[m] = (uint16_t)bits;
      }
      n--;
    }
  }
}

DFL_HD inline void build_tree(Cold& s, Tree& tr) {
  uint16_t* fc = tr.fc;
  uint16_t* dl = tr.dl;
  uint16_t* heap = s.a->heap;
  uint8_t* depth = s.a->depth;
  const int elems = tr.elems;
  int max_code = -1, node;
  int heap_len = 0, heap_max = kHeapSize;
  for (int n = 0; n < elems; n++) {
    if (fc[n] != 0) {
      heap[++heap_len] = (uint16_t)(max_code = n);
      depth[n] = 0;
    } else {
      dl[n] = 0;
    }
  }
  while (heap_len < 2) {
    node = heap[++heap_len] = (uint16_t)(max_code < 2 ? ++max_code : 0);
    fc[node] = 1;
    depth[node] = 0;
    s.opt_len--;
    if (tr.slen) s.static_len -= tr.slen[node];
  }
  tr.max_code = max_code;
  for (int n = heap_len / 2; n >= 1; n--) pqdownheap(s, fc, n, heap_len);
  node = elems;
  do {
    int n = heap[1];
    heap[1] = heap[heap_len--];
    pqdownheap(s, fc, 1, heap_len);
    int m = heap[1];
    heap[--heap_max] = (uint16_t)n;
    heap[--heap_max] = (uint16_t)m;
    fc[node] = (uint16_t)(fc[n] + fc[m]);
    depth[node] = (uint8_t)((depth[n] >= depth[m] ? depth[n] : depth[m]) + 1);
    dl[n] = dl[m] = (uint16_t)node;
    heap[1] = (uint16_t)(node++);
    pqdownheap(s, fc, 1, heap_len);
  } while (heap_len >= 2);
  heap[--heap_max] = heap[1];
  gen_bitlen(s, tr, heap_max);
  // gen_codes over dl (lengths, <= 15 here) -> fc (codes)
  uint16_t next_code[kMaxBits + 1];
  unsigned code = 0;
  for (int bits = 1; bits <= kMaxBits; bits++) {
    code = (code + s.a->bl_count[bits - 1]) << 1;
    next_code[bits] = (uint16_t)code;
  }
  for (int n = 0; n <= max_code; n++) {
    int len = dl[n];
    if (len == 0) continue;
    fc[n] = (uint16_t)bi_reverse(next_code[len]++, len);
  }
}

DFL_HD inline void scan_tree(Cold& s, Tree& tr, int max_code) {
  uint16_t* dl = tr.dl;
  uint16_t* bfc = s.b.fc;
  int prevlen = -1, curlen, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  dl[max_code + 1] = 0xffff;  // guard
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = dl[n + 1];
    if (++count < max_count && curlen == nextlen) continue;
    else if (count < min_count) bfc[curlen] += count;
    else if (curlen != 0) {
      if (curlen != prevlen) bfc[curlen]++;
      bfc[16]++;
    } else if (count <= 10) bfc[17]++;
    else bfc[18]++;
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

DFL_HD inline void send_code(Cold& s, int c, const uint16_t* codes, const uint16_t* lens) {
  s.out.bits(codes[c], lens[c]);
}

DFL_HD inline void send_tree(Cold& s, Tree& tr, int max_code) {
  uint16_t* dl = tr.dl;
  int prevlen = -1, curlen, nextlen = dl[0], count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  for (int n = 0; n <= max_code; n++) {
    curlen = nextlen;
    nextlen = dl[n + 1];
    if (++count < max_count && curlen == nextlen) continue;
    else if (count < min_count) {
      do {
        send_code(s, curlen, s.b.fc, s.b.dl);
      } while (--count != 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        send_code(s, curlen, s.b.fc, s.b.dl);
        count--;
      }
      send_code(s, 16, s.b.fc, s.b.dl);
      s.out.bits(count - 3, 2);
    } else if (count <= 10) {
      send_code(s, 17, s.b.fc, s.b.dl);
      s.out.bits(count - 3, 3);
    } else {
      send_code(s, 18, s.b.fc, s.b.dl);
      s.out.bits(count - 11, 7);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

DFL_HD inline int d_code(const Tables* t, unsigned dist) {
  return dist < 256 ? t->dist_code[dist] : t->dist_code[256 + (dist >> 7)];
}

template <typename CodeT, typename LenT>
DFL_HD inline void compress_block(Cold& s, const CodeT* lcode, const LenT* llen, const CodeT* dcode,
                                  const LenT* dlen) {
  const Tables* t = s.t;
  unsigned lx = 0;
  if (s.last_lit != 0) do {
      unsigned dist = s.a->d_buf[lx];
      int lc = s.a->l_buf[lx++];
      if (dist == 0) {
        s.out.bits(lcode[lc], llen[lc]);
      } else {
        int code = t->length_code[lc];
        s.out.bits(lcode[code + kLiterals + 1], llen[code + kLiterals + 1]);
        int extra = extra_lbits(code);
        if (extra != 0) s.out.bits((unsigned)(lc - t->base_length[code]), extra);
        dist--;
        code = d_code(t, dist);
        s.out.bits(dcode[code], dlen[code]);
        extra = extra_dbits(code);
        if (extra != 0) s.out.bits(dist - (unsigned)t->base_dist[code], extra);
      }
    } while (lx < s.last_lit);
  s.out.bits(lcode[kEndBlock], llen[kEndBlock]);
}

// _tr_flush_block (trees.c), level > 0
DFL_HD DFL_NOINLINE void flush_block(Cold& s, bool has_buf, uint32_t buf_start, uint32_t stored_len, int last) {
  build_tree(s, s.l);
  build_tree(s, s.d);
  // build_bl_tree
  scan_tree(s, s.l, s.l.max_code);
  scan_tree(s, s.d, s.d.max_code);
  build_tree(s, s.b);
  int max_blindex;
  for (max_blindex = kBlCodes - 1; max_blindex >= 3; max_blindex--)
    if (s.b.dl[bl_order(max_blindex)] != 0) break;
  s.opt_len += 3 * ((uint32_t)max_blindex + 1) + 5 + 5 + 4;
  uint32_t opt_lenb = (s.opt_len + 3 + 7) >> 3;
  uint32_t static_lenb = (s.static_len + 3 + 7) >> 3;
  if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
  if (stored_len + 4 <= opt_lenb && has_buf) {
    // _tr_stored_block
    s.out.bits((0 << 1) + last, 3);
    s.out.windup();
    s.out.byte((uint8_t)stored_len);
    s.out.byte((uint8_t)(stored_len >> 8));
    s.out.byte((uint8_t)~stored_len);
    s.out.byte((uint8_t)(~stored_len >> 8));
    for (uint32_t i = 0; i < stored_len; ++i) s.out.byte(s.win(buf_start + i));
  } else if (static_lenb == opt_lenb) {
    s.out.bits((1 << 1) + last, 3);
    compress_block(s, s.t->sl_code, s.t->sl_len, s.t->sd_code, s.t->sd_len);
  } else {
    const int lcodes = s.l.max_code + 1, dcodes = s.d.max_code + 1, blcodes = max_blindex + 1;
    s.out.bits((2 << 1) + last, 3);
    s.out.bits(lcodes - 257, 5);
    s.out.bits(dcodes - 1, 5);
    s.out.bits(blcodes - 4, 4);
    for (int rank = 0; rank < blcodes; rank++) s.out.bits(s.b.dl[bl_order(rank)], 3);
    send_tree(s, s.l, lcodes - 1);
    send_tree(s, s.d, dcodes - 1);
    compress_block(s, s.l.fc, s.l.dl, s.d.fc, s.d.dl);
  }
  init_block(s);
  if (last) s.out.windup();
}

// 8 bytes at any address (device: two aligned loads + funnel shift; the
// buffers carry >= 16 bytes of padding past the last payload)
DFL_HD inline uint64_t ld8(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uintptr_t a = (uintptr_t)p;
  const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
  const unsigned sh = (unsigned)(a & 7) * 8;
  const uint64_t lo = q[0];
  return sh ? (lo >> sh) | (q[1] << (64 - sh)) : lo;
#else
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
#endif
}

DFL_HD inline uint32_t longest_match(State& s, uint32_t cur_match) {
  unsigned chain_length = s.cfg.chain;
  const uint32_t scan = s.strstart;
  int best_len = (int)s.prev_length;
  int nice_match = s.cfg.nice;
  const uint32_t limit = s.strstart > (uint32_t)kMaxDist ? s.strstart - kMaxDist : 0;
  uint8_t scan_end1 = s.win(scan + best_len - 1);
  uint8_t scan_end = s.win(scan + best_len);
  if (s.prev_length >= s.cfg.good) chain_length >>= 2;
  if ((uint32_t)nice_match > s.lookahead) nice_match = (int)s.lookahead;
  const uint8_t s0 = s.win(scan), s1 = s.win(scan + 1);
  const bool fast = !s.w.slid && scan + kMaxMatch + 1 <= s.w.len;
  uint32_t next;
  do {
    const uint32_t match = cur_match;
    // the next chain link does not depend on this candidate: load it first so
    // its miss overlaps the candidate's window reads
    next = s.a->prev[cur_match & kWMask];
    if (fast) {  // all four bytes in the payload: issue the loads together
      const uint8_t* pm = s.w.in + match;
      const uint32_t m0 = pm[best_len], m1 = pm[best_len - 1], m2 = pm[0], m3 = pm[1];
      if ((m0 ^ scan_end) | (m1 ^ scan_end1) | (m2 ^ s0) | (m3 ^ s1)) continue;
    } else if (s.win(match + best_len) != scan_end || s.win(match + best_len - 1) != scan_end1 ||
               s.win(match) != s0 || s.win(match + 1) != s1) {
      continue;
    }
    // scan[2] == match[2] is assumed (equal hash, HASH_BITS >= 8)
    int len = 3;
    if (fast) {  // bytes 3..258 of both strings inside the payload, no remap
      const uint8_t* ps = s.w.in + scan;
      const uint8_t* pm = s.w.in + match;
      for (;;) {
        const uint64_t x = ld8(ps + len) ^ ld8(pm + len);
        if (x) {
          len += (int)(__builtin_ctzll(x) >> 3);
          break;
        }
        len += 8;
        if (len >= kMaxMatch) break;
      }
      if (len > kMaxMatch) len = kMaxMatch;
    } else {
      while (len < kMaxMatch && s.win(scan + len) == s.win(match + len)) len++;
    }
    if (len > best_len) {
      s.match_start = cur_match;
      best_len = len;
      if (len >= nice_match) break;
      scan_end1 = s.win(scan + best_len - 1);
      scan_end = s.win(scan + best_len);
    }
  } while ((cur_match = next) > limit && --chain_length != 0);
  if ((uint32_t)best_len <= s.lookahead) return (uint32_t)best_len;
  return s.lookahead;
}

DFL_HD inline bool tally_lit(State& s, uint8_t c) {
  s.a->d_buf[s.last_lit] = 0;
  s.a->l_buf[s.last_lit++] = c;
  s.a->lfc[c]++;
  return s.last_lit == kLitBufSize - 1;
}
DFL_HD inline bool tally_dist(State& s, unsigned dist, unsigned len) {
  s.a->d_buf[s.last_lit] = (uint16_t)dist;
  s.a->l_buf[s.last_lit++] = (uint8_t)len;
  dist--;
  s.a->lfc[s.t->length_code[len] + kLiterals + 1]++;
  s.a->dfc[d_code(s.t, dist)]++;
  return s.last_lit == kLitBufSize - 1;
}

DFL_HD inline void flush(State& s, int last) {
  const bool has = s.block_start >= 0;
  s.c->w = s.w;
  s.c->last_lit = s.last_lit;
  s.last_lit = 0;
  flush_block(*s.c, has, has ? (uint32_t)s.block_start : 0, (uint32_t)((int32_t)s.strstart - s.block_start), last);
  s.block_start = (int32_t)s.strstart;
}

// slide_hash: every Pos m -> m >= wsize ? m - wsize : NIL, four per word
DFL_HD inline void slide_words(uint64_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i) {
    uint64_t v = w[i], r = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t m = (uint32_t)(v >> (16 * k)) & 0xffff;
      r |= (uint64_t)(m >= (uint32_t)kWSize ? m - kWSize : 0) << (16 * k);
    }
    w[i] = r;
  }
}

// fill_window after the first read: only the slide can happen
DFL_HD inline void fill_window(State& s) {
  if (s.strstart >= (uint32_t)(kWSize + kMaxDist)) {
    s.w.slid = true;  // [wsize, len) moved to [0, len - wsize)
    s.match_start -= kWSize;
    s.strstart -= kWSize;
    s.block_start -= kWSize;
    slide_words(reinterpret_cast<uint64_t*>(s.a->head), kHashSize / 4);
    slide_words(reinterpret_cast<uint64_t*>(s.a->prev), kWSize / 4);
  }
}

// deflate(Z_FINISH) of in[0, len) on a reset stream; returns the compressed
// size; *overflow when it does not fit cap (htsjdk: deflater not finished).
// head_cleared: the caller already zeroed a->head (lm_init's CLEAR_HASH).
DFL_HD inline uint32_t deflate_block(Arena* a, const Tables* t, int level, const uint8_t* in, uint32_t len,
                                     uint8_t* out, uint32_t cap, bool* overflow, bool head_cleared = false) {
  State s;
  Cold c;
  s.w.in = in;
  s.w.len = len;
  s.w.slid = false;
  s.w.copied = len > (uint32_t)kWSize ? len - kWSize : 0;
  s.a = a;
  s.t = t;
  s.c = &c;
  s.cfg = level_config(level);
  c.a = a;
  c.t = t;
  c.w = s.w;
  c.l = Tree{a->lfc, a->ldl, t->sl_len, 0, kLCodes, kMaxBits, kLiterals + 1, 0};
  c.d = Tree{a->dfc, a->ddl, t->sd_len, 1, kDCodes, kMaxBits, 0, 0};
  c.b = Tree{a->bfc, a->bdl, nullptr, 2, kBlCodes, kMaxBlBits, 0, 0};
  c.out = Out{out, cap, 0, 0, 0, false};
  // lm_init: CLEAR_HASH (prev is not cleared by zlib; stale entries are never reached)
  if (!head_cleared)
    for (int n = 0; n < kHashSize; ++n) a->head[n] = 0;
  s.strstart = 0;
  s.block_start = 0;
  s.lookahead = 0;
  s.match_length = s.prev_length = kMinMatch - 1;
  s.match_available = 0;
  s.match_start = 0;
  s.prev_match = 0;
  s.ins_h = 0;
  s.last_lit = 0;
  init_block(c);
  // first fill_window: the whole payload is read
  s.lookahead = len;
  if (s.lookahead >= (uint32_t)kMinMatch) {
    s.ins_h = s.win(0);
    s.ins_h = ((s.ins_h << kHashShift) ^ s.win(1)) & kHashMask;
  }
  if (level <= 3) {
    // deflate_fast: no lazy evaluation; max_insert_length = max_lazy
    for (;;) {
      if (s.lookahead < (uint32_t)kMinLookahead) {
        fill_window(s);
        if (s.lookahead == 0) break;
      }
      uint32_t hash_head = 0;
      if (s.lookahead >= (uint32_t)kMinMatch) insert_string(s, s.strstart, &hash_head);
      if (hash_head != 0 && s.strstart - hash_head <= (uint32_t)kMaxDist) s.match_length = longest_match(s, hash_head);
      bool bflush;
      if (s.match_length >= (uint32_t)kMinMatch) {
        bflush = tally_dist(s, s.strstart - s.match_start, s.match_length - kMinMatch);
        s.lookahead -= s.match_length;
        if (s.match_length <= s.cfg.lazy && s.lookahead >= (uint32_t)kMinMatch) {
          s.match_length--;
          do {
            s.strstart++;
            insert_string(s, s.strstart, &hash_head);
          } while (--s.match_length != 0);
          s.strstart++;
        } else {
          s.strstart += s.match_length;
          s.match_length = 0;
          s.ins_h = s.win(s.strstart);
          s.ins_h = ((s.ins_h << kHashShift) ^ s.win(s.strstart + 1)) & kHashMask;
        }
      } else {
        bflush = tally_lit(s, s.win(s.strstart));
        s.lookahead--;
        s.strstart++;
      }
      if (bflush) flush(s, 0);
    }
    flush(s, 1);
    *overflow = c.out.overflow || c.out.n >= cap;
    return c.out.n;
  }
  // deflate_slow
  for (;;) {
    if (s.lookahead < (uint32_t)kMinLookahead) {
      fill_window(s);
      if (s.lookahead == 0) break;
    }
    uint32_t hash_head = 0;
    if (s.lookahead >= (uint32_t)kMinMatch) insert_string(s, s.strstart, &hash_head);
    s.prev_length = s.match_length, s.prev_match = s.match_start;
    s.match_length = kMinMatch - 1;
    if (hash_head != 0 && s.prev_length < s.cfg.lazy && s.strstart - hash_head <= (uint32_t)kMaxDist) {
      s.match_length = longest_match(s, hash_head);
      if (s.match_length <= 5 && (s.match_length == kMinMatch && s.strstart - s.match_start > (uint32_t)kTooFar))
        s.match_length = kMinMatch - 1;
    }
    if (s.prev_length >= (uint32_t)kMinMatch && s.match_length <= s.prev_length) {
      const uint32_t max_insert = s.strstart + s.lookahead - kMinMatch;
      const bool bflush = tally_dist(s, s.strstart - 1 - s.prev_match, s.prev_length - kMinMatch);
      s.lookahead -= s.prev_length - 1;
      s.prev_length -= 2;
      do {
        if (++s.strstart <= max_insert) insert_string(s, s.strstart, &hash_head);
      } while (--s.prev_length != 0);
      s.match_available = 0;
      s.match_length = kMinMatch - 1;
      s.strstart++;
      if (bflush) flush(s, 0);
    } else if (s.match_available) {
      const bool bflush = tally_lit(s, s.win(s.strstart - 1));
      if (bflush) flush(s, 0);
      s.strstart++;
      s.lookahead--;
    } else {
      s.match_available = 1;
      s.strstart++;
      s.lookahead--;
    }
  }
  if (s.match_available) {
    tally_lit(s, s.win(s.strstart - 1));
    s.match_available = 0;
  }
  flush(s, 1);
  *overflow = c.out.overflow || c.out.n >= cap;
  return c.out.n;
}

}  // namespace dfl
}  // namespace hbam
