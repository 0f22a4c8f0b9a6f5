// sync_sim.c -- host model of phase A's slice self-synchronisation
// (developer probe, not product).  For every dynamic DEFLATE block of the
// first BGZF blocks of a BAM: walk the true symbol path (literal pairs as the
// GPU's 10-bit root table forms them), cut the stream into 256 slices and, for
// warm-up lengths d, start each slice's walk d bits before its nominal start.
// A slice "matches" when the first boundary of its walk at or past its nominal
// start is the first TRUE boundary there (its predecessor's exit when the
// predecessor is on the true path).  Prints per d: the lane mismatch rate, the
// share of 64-lane waves holding a mismatch, and the warm-up symbols paid.
// Build: gcc -O2 -o scripts/bin/sync_sim scripts/sync_sim.c
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const uint16_t LB[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LE[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t DE[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t CLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int g_pair = 1;
static const uint8_t* g_buf;
static uint64_t g_nbits;
static uint32_t bits(uint64_t p, int n) {  // n <= 24, LSB first
  uint32_t v = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t q = p + i;
    uint32_t b = q < g_nbits ? (g_buf[q >> 3] >> (q & 7)) & 1 : 0;
    v |= b << i;
  }
  return v;
}

// canonical code: table of (symbol, length) indexed by reversed 15-bit code
typedef struct {
  int16_t sym[1 << 15];
  uint8_t len[1 << 15];
} Code;
static int build(Code* c, const uint8_t* lens, int n) {
  int cnt[16] = {0}, next[16];
  for (int i = 0; i < n; ++i) cnt[lens[i]]++;
  cnt[0] = 0;
  int code = 0;
  for (int l = 1; l < 16; ++l) {
    code = (code + cnt[l - 1]) << 1;
    next[l] = code;
  }
  memset(c->len, 0, sizeof c->len);
  for (int s = 0; s < n; ++s) {
    int l = lens[s];
    if (!l) continue;
    int cd = next[l]++;
    int rev = 0;
    for (int i = 0; i < l; ++i) rev |= ((cd >> i) & 1) << (l - 1 - i);
    for (int r = rev; r < (1 << 15); r += 1 << l) {
      c->sym[r] = s;
      c->len[r] = l;
    }
  }
  return 0;
}
static Code LIT, DIST, CL;

// one GPU symbol at p: returns bits consumed (0 = invalid / EOB); *eob set on EOB
static int step(uint64_t p, int* eob) {
  *eob = 0;
  uint32_t b = bits(p, 15);
  int l1 = LIT.len[b];
  if (!l1) return 0;
  int s = LIT.sym[b];
  if (s < 256) {
    if (g_pair && l1 < 10) {  // pair when the next literal code fits the 10-bit root too
      uint32_t b2 = bits(p + l1, 15);
      int l2 = LIT.len[b2];
      if (l2 && LIT.sym[b2] < 256 && l1 + l2 <= 10) return l1 + l2;
    }
    return l1;
  }
  if (s == 256) {
    *eob = 1;
    return l1;
  }
  if (s > 285) return 0;
  int n = l1 + LE[s - 257];
  uint32_t d = bits(p + n, 15);
  int dl = DIST.len[d];
  if (!dl || DIST.sym[d] >= 30) return 0;
  return n + dl + DE[DIST.sym[d]];
}

#define NDELTA 9
static const int DELTAS[NDELTA] = {0, 16, 32, 48, 64, 96, 128, 192, 256};
static uint64_t lanes = 0, mism[NDELTA], waves = 0, wmism[NDELTA], warm_syms[NDELTA], slice_syms = 0;
static uint64_t blocks_seen = 0;

static void sim_sync(uint64_t b0, uint64_t bend, const uint8_t* tb);
static void sim_block(uint64_t b0, uint64_t bend) {
  // true boundaries
  uint64_t R = bend - b0;
  uint8_t* tb = calloc((R + 64) / 8 + 1, 1);
  uint64_t p = b0;
  uint64_t nsym = 0;
  for (;;) {
    int eob, n = step(p, &eob);
    tb[(p - b0) >> 3] |= 1 << ((p - b0) & 7);
    if (!n || eob) break;
    p += n;
    ++nsym;
  }
  uint64_t S = (R + 255) / 256;
  // first true boundary >= a
  uint64_t* ft = malloc(sizeof(uint64_t) * 256);
  for (int l = 0; l < 256; ++l) {
    uint64_t a = b0 + l * S;
    uint64_t q = a;
    while (q < bend && !((tb[(q - b0) >> 3] >> ((q - b0) & 7)) & 1)) ++q;
    ft[l] = q;
  }
  slice_syms += nsym;
  for (int w = 0; w < 4; ++w) {
    int wm[NDELTA] = {0};
    for (int l = w * 64; l < w * 64 + 64; ++l) {
      if (l == 0) continue;
      uint64_t a = b0 + l * S;
      if (a >= bend) continue;
      ++lanes;
      for (int k = 0; k < NDELTA; ++k) {
        uint64_t q = a >= b0 + DELTAS[k] ? a - DELTAS[k] : b0;
        uint64_t ws = 0;
        while (q < a) {
          int eob, n = step(q, &eob);
          if (!n || eob) { q = ~0ull; break; }
          q += n;
          ++ws;
        }
        warm_syms[k] += ws;
        if (q != ft[l]) {
          mism[k]++;
          wm[k] = 1;
        }
      }
    }
    waves++;
    for (int k = 0; k < NDELTA; ++k) wmism[k] += wm[k];
  }
  sim_sync(b0, bend, tb);
  free(ft);
  free(tb);
}


#define NSET 4
static const char* SETN[NSET] = {"4,8,16,32", "every 4 to 32", "every 4 to 64", "every boundary"};
static double set_wave_cost[NSET], set_lane_cost[NSET], slice_cost_sum = 0;
static uint64_t set_waves = 0, set_lanes = 0;
static int in_set(int k, int sym) {  // sym = 1-based symbol count of the spec walk at a boundary
  if (k == 0) return sym == 4 || sym == 8 || sym == 16 || sym == 32;
  if (k == 1) return sym % 4 == 0 && sym <= 32;
  if (k == 2) return sym % 4 == 0 && sym <= 64;
  return 1;
}
static void sim_sync(uint64_t b0, uint64_t bend, const uint8_t* tb) {
  uint64_t R = bend - b0, S = (R + 255) / 256;
  static uint64_t bpos[4096];
  static uint8_t bset[4096];
  for (int w = 0; w < 4; ++w) {
    double wmax[NSET] = {0};
    for (int l = w * 64; l < w * 64 + 64; ++l) {
      uint64_t a = b0 + l * S, stop = a + S;
      if (a >= bend) continue;
      if (stop > bend) stop = bend;
      // spec walk from a to stop: boundary after each symbol
      int ns = 0;
      uint64_t q = a;
      while (q < stop && ns < 4096) {
        int eob, n = step(q, &eob);
        if (!n || eob) break;
        q += n;
        bpos[ns++] = q;
      }
      // true start: first true boundary >= a
      uint64_t t = a;
      while (t < bend && !((tb[(t - b0) >> 3] >> ((t - b0) & 7)) & 1)) ++t;
      // symbols of the true walk (slice) for the full-slice cost
      int full = 0;
      { uint64_t z = t; while (z < stop) { int eob, n = step(z, &eob); if (!n || eob) break; z += n; ++full; } }
      slice_cost_sum += full;
      for (int k = 0; k < NSET; ++k) {
        // sync walk from t: count symbols until its position equals a checkpoint boundary of the spec walk
        uint64_t z = t;
        int c = 0, merged = 0;
        int j = 0;
        while (z < stop) {
          while (j < ns && bpos[j] < z) ++j;
          if (j < ns && bpos[j] == z && in_set(k, j + 1)) { merged = 1; break; }
          int eob, n = step(z, &eob);
          if (!n || eob) break;
          z += n;
          ++c;
        }
        (void)merged;
        set_lane_cost[k] += c;
        if (c > wmax[k]) wmax[k] = c;
      }
      ++set_lanes;
    }
    for (int k = 0; k < NSET; ++k) set_wave_cost[k] += wmax[k];
    ++set_waves;
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int maxb = argc > 2 ? atoi(argv[2]) : 200;
  g_pair = argc > 3 ? atoi(argv[3]) : 1;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* d = malloc(sz);
  if (fread(d, 1, sz, f) != (size_t)sz) return 1;
  long off = 0;
  int nb = 0;
  while (off + 18 <= sz && nb < maxb) {
    int bsize = (d[off + 16] | (d[off + 17] << 8)) + 1;
    const uint8_t* cd = d + off + 18;
    uint64_t clen = bsize - 26;
    g_buf = cd;
    g_nbits = clen * 8;
    uint64_t p = 0;
    ++nb;
    for (;;) {
      if (p + 3 > g_nbits) break;
      uint32_t h = bits(p, 3);
      p += 3;
      int fin = h & 1, type = h >> 1;
      if (type != 2) break;  // C2: dynamic blocks only
      int hlit = bits(p, 5) + 257, hdist = bits(p + 5, 5) + 1, hclen = bits(p + 10, 4) + 4;
      p += 14;
      uint8_t cl[19] = {0};
      for (int i = 0; i < hclen; ++i, p += 3) cl[CLO[i]] = bits(p, 3);
      build(&CL, cl, 19);
      uint8_t lens[320] = {0};
      int n = 0;
      while (n < hlit + hdist) {
        uint32_t b = bits(p, 15);
        int s = CL.sym[b];
        p += CL.len[b];
        if (s < 16) lens[n++] = s;
        else if (s == 16) { int r = 3 + bits(p, 2); p += 2; for (int i = 0; i < r; ++i, ++n) lens[n] = lens[n - 1]; }
        else if (s == 17) { int r = 3 + bits(p, 3); p += 3; n += r; }
        else { int r = 11 + bits(p, 7); p += 7; n += r; }
      }
      build(&LIT, lens, hlit);
      build(&DIST, lens + hlit, hdist);
      // true walk to EOB
      uint64_t q = p;
      for (;;) {
        int eob, k = step(q, &eob);
        if (!k) { fprintf(stderr, "bad symbol\n"); return 1; }
        q += k;
        if (eob) break;
      }
      sim_block(p, q);
      ++blocks_seen;
      p = q;
      if (fin) break;
    }
    off += bsize;
  }
  printf("deflate blocks %llu, lanes %llu, symbols per slice %.1f\n", (unsigned long long)blocks_seen,
         (unsigned long long)lanes, (double)slice_syms / (blocks_seen * 256.0));
  for (int k = 0; k < NDELTA; ++k)
    printf("warm-up %3d bits: lane mismatch %.4f  waves with a mismatch %.4f  warm-up symbols/lane %.1f\n", DELTAS[k],
           (double)mism[k] / lanes, (double)wmism[k] / waves, (double)warm_syms[k] / lanes);
  printf("true-walk symbols per slice %.1f\n", slice_cost_sum / set_lanes);
  for (int k = 0; k < NSET; ++k)
    printf("sync checkpoints %-16s mean lane walk %.1f symbols, mean wave max %.1f\n", SETN[k],
           set_lane_cost[k] / set_lanes, set_wave_cost[k] / set_waves);
  return 0;
}
// (appended) -- see main2: sync-walk cost model with checkpoint sets
