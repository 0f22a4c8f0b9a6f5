// dual_sim.c -- host model of phase A with 256 or 512 slices per DEFLATE
// block (developer probe, not product; symbol walk and true path as in
// sync_sim.c).  Per 64-lane wave (each lane walking NS/256 slices in
// lockstep): the speculative walk's length (max over the wave), then every
// sync iteration until no exit changes (a slice re-walks from its
// predecessor's latest exit until it meets a boundary of its speculative walk
// at symbols mf, 2mf, 4mf, 8mf -- mf = 2 under 400 bits -- or passes its
// stop), each costing the wave's longest re-walk; emit = spec.
// NOTE: the "2nd" row is the second DEFLATE block of a BGZF block's chunk
// order as the kernel's round 0 sees it, "1st" the first (labels as printed).
// Build: gcc -O2 -o scripts/bin/dual_sim scripts/dual_sim.c
// Run:   scripts/bin/dual_sim <C2-like BAM> [BGZF blocks] [256|512]
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



static int NSL = 256;  // slices per DEFLATE block
static double sp_cost[2], sy_cost[2], nwaves[2], sym_tot[2], iters[2], nblk[2];
static int cur_round = 0;
static int walkn(uint64_t g, uint64_t stop, uint64_t* pos, int cap) {
  int n = 0; uint64_t q = g;
  while (q < stop && n < cap) { int eob, k = step(q, &eob); if (!k || eob) break; q += k; pos[n++] = q; }
  return n;
}
// walk from g: symbols until reaching a checkpoint of the spec walk (merge) or
// passing stop; returns symbols walked, *ex = exit (first boundary >= stop)
static int sync_walk(uint64_t g, uint64_t stop, const uint64_t* sp, int ns, int mf, uint64_t sx, uint64_t* ex) {
  uint64_t q = g; int n = 0;
  for (;;) {
    for (int m = mf; m <= 8 * mf; m *= 2) if (m <= ns && sp[m - 1] == q) { *ex = sx; return n; }
    if (q >= stop) { *ex = q; return n; }
    int eob, k = step(q, &eob);
    if (!k || eob) { *ex = q; return n; }
    q += k; ++n;
  }
}
static uint64_t SPP[1024][4096];
static void sim_sync(uint64_t b0, uint64_t bend, const uint8_t* tb) {
  uint64_t R = bend - b0, S = (R + NSL - 1) / NSL;
  int mf = S < 400 ? 2 : 4;
  static int ns[1024], lenspec[1024], cost[1024];
  static uint64_t a_[1024], st[1024], sx[1024], ex[1024], prevx[1024];
  int nsl = 0;
  for (int sl = 0; sl < NSL; ++sl) {
    a_[sl] = b0 + sl * S; st[sl] = a_[sl] + S;
    if (a_[sl] >= bend) break;
    if (st[sl] > bend) st[sl] = bend;
    ns[sl] = walkn(a_[sl], st[sl], SPP[sl], 4096);
    sx[sl] = ns[sl] ? SPP[sl][ns[sl] - 1] : a_[sl];
    // the spec walk's exit: the first boundary >= stop (walkn stops there)
    ex[sl] = sx[sl];
    lenspec[sl] = ns[sl];
    nsl = sl + 1;
  }
  int per = NSL / 256;
  // spec cost per wave
  for (int w = 0; w < 4; ++w) {
    int m = 0;
    for (int l = w * 64; l < w * 64 + 64; ++l) for (int k = 0; k < per; ++k) { int sl = l + 256 * k; if (sl < nsl && lenspec[sl] > m) m = lenspec[sl]; }
    sp_cost[cur_round] += m; nwaves[cur_round] += 1;
  }
  // sync iterations: slice i (> 0) re-walks from ex[i-1] when it differs from where its walk started
  static uint64_t start[1024];
  for (int sl = 0; sl < nsl; ++sl) start[sl] = a_[sl];
  int it = 0;
  for (;;) {
    int any = 0;
    for (int sl = 0; sl < nsl; ++sl) prevx[sl] = ex[sl];
    for (int sl = 0; sl < nsl; ++sl) cost[sl] = 0;
    for (int sl = 1; sl < nsl; ++sl) {
      uint64_t px = prevx[sl - 1];
      if (px == start[sl]) continue;
      any = 1;
      start[sl] = px;
      uint64_t e;
      cost[sl] = sync_walk(px, st[sl], SPP[sl], ns[sl], mf, sx[sl], &e);
      ex[sl] = e;
    }
    if (!any || ++it > 40) break;
    for (int w = 0; w < 4; ++w) {
      int m = 0;
      for (int l = w * 64; l < w * 64 + 64; ++l) for (int k = 0; k < per; ++k) { int sl = l + 256 * k; if (sl < nsl && cost[sl] > m) m = cost[sl]; }
      sy_cost[cur_round] += m;
    }
    iters[cur_round] += 1;
  }
  nblk[cur_round] += 1;
  for (int sl = 0; sl < nsl; ++sl) sym_tot[cur_round] += lenspec[sl];
}
int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int maxb = argc > 2 ? atoi(argv[2]) : 200;
  NSL = argc > 3 ? atoi(argv[3]) : 256;
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
      cur_round = (p == 0 || cur_round == 1) ? 0 : 1;
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
  for (int r = 0; r < 2; ++r)
    printf("DEFLATE block %s, %d slices: per wave spec %.1f  sync (all iterations) %.1f  emit %.1f  total %.1f; "
           "sync iterations per block %.2f, symbols/slice %.1f\n", r ? "1st" : "2nd", NSL, sp_cost[r] / nwaves[r],
           sy_cost[r] / nwaves[r], sp_cost[r] / nwaves[r], (2 * sp_cost[r] + sy_cost[r]) / nwaves[r],
           iters[r] / nblk[r], sym_tot[r] / (nblk[r] * NSL));
  return 0;
}
// (appended) -- see main2: sync-walk cost model with checkpoint sets
