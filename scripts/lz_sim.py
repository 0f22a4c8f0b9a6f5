"""Host model of phase B's resolve step (k_inflate_lz77 step 4) on C2-like
blocks: the LZ77 tokens of real zlib streams (a small DEFLATE token decoder
below), the u16 map as step 3 leaves it, and the chase schedules compared in
LDS operations per wave (the quantity the resolve's time follows):
  lockstep  the kernel today: each thread chases kLzChase = 2 positions 1024
            apart per iteration, a wave steps until its deepest chase ends
  dynamic   each lane slot takes the wave's next position as soon as its
            chase ends (ballot / mbcnt hand-out, no lockstep per iteration)
Path compression (pointer jumping) is modelled at the granularity of one
iteration of all 16 waves: positions of earlier iterations are resolved.
usage: python scripts/lz_sim.py [records] [blocks]"""
import os
import sys
import zlib

import numpy as np

for _d in ("hadoop-bam_amd", "oracle"):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", _d))

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227,
         258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
         6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class Bits:
    def __init__(self, b):
        self.v = int.from_bytes(b, "little")
        self.p = 0

    def get(self, n):
        r = (self.v >> self.p) & ((1 << n) - 1)
        self.p += n
        return r


def huff(lens):
    """canonical code -> {(len, code): symbol}"""
    mx = max(lens) if lens else 0
    cnt = [0] * (mx + 1)
    for l in lens:
        if l:
            cnt[l] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + cnt[b - 1]) << 1
        nxt[b] = code
    t = {}
    for s, l in enumerate(lens):
        if l:
            t[(l, nxt[l])] = s
            nxt[l] += 1
    return t, mx


def sym(bits, t):
    code, l = 0, 0
    while True:
        code = (code << 1) | bits.get(1)
        l += 1
        if (l, code) in t:
            return t[(l, code)]


def tokens(raw):
    """(is_match, value_or_len, dist) tokens of a raw DEFLATE stream"""
    bits = Bits(raw)
    out = []
    while True:
        final = bits.get(1)
        typ = bits.get(2)
        if typ == 0:
            raise ValueError("stored block")
        if typ == 1:
            ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
            dl = [5] * 30
        else:
            hlit, hdist, hclen = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
            order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
            cl = [0] * 19
            for i in range(hclen):
                cl[order[i]] = bits.get(3)
            ct, _ = huff(cl)
            lens = []
            while len(lens) < hlit + hdist:
                s = sym(bits, ct)
                if s < 16:
                    lens.append(s)
                elif s == 16:
                    lens += [lens[-1]] * (3 + bits.get(2))
                elif s == 17:
                    lens += [0] * (3 + bits.get(3))
                else:
                    lens += [0] * (11 + bits.get(7))
            ll, dl = lens[:hlit], lens[hlit:]
        lt, _ = huff(ll)
        dt, _ = huff(dl)
        while True:
            s = sym(bits, lt)
            if s < 256:
                out.append((0, s, 0))
            elif s == 256:
                break
            else:
                i = s - 257
                ln = LBASE[i] + bits.get(LEXT[i])
                d = sym(bits, dt)
                dist = DBASE[d] + bits.get(DEXT[d])
                out.append((1, ln, dist))
        if final:
            return out


def source_map(toks, isize):
    """src[p] = -1 for a literal position, else the position its byte comes from"""
    src = np.full(isize, -1, np.int64)
    p = 0
    for m, a, d in toks:
        if m:
            n = min(a, isize - p)
            src[p:p + n] = np.arange(p, p + n) - d
            p += n
        else:
            p += 1
    return src


def depths(src):
    """hops from each position to a literal without compression"""
    d = np.zeros(len(src), np.int64)
    for p in range(len(src)):
        s = src[p]
        d[p] = 0 if s < 0 else d[s] + 1
    return d


def simulate(src, lanes=64, waves=16, chase=2):
    """wave-steps of the resolve per wave (each step = chase reads + chase
    stores per lane), both schedules with positions before the current
    2048-position stretch resolved (the kernel's path compression)."""
    n = len(src)
    nthr = lanes * waves
    per_it = chase * nthr
    h = np.zeros(n, np.int64)
    for p in range(n):
        lo = p - p % per_it
        q, k = p, 0
        while src[q] >= lo:
            q = src[q]
            k += 1
        h[p] = k
    lock = np.zeros(waves)
    for base in range(0, n, per_it):
        for w in range(waves):
            mx = 0
            for k in range(chase):
                lo = base + k * nthr + w * lanes
                if lo < n:
                    mx = max(mx, int(h[lo:min(n, lo + lanes)].max()))
            lock[w] += 1 + mx
    dyn = np.zeros(waves)
    for w in range(waves):
        ks = [1024 * (k >> 6) + 64 * w + (k & 63) for k in range((n + 1023) // 1024 * 64)]
        cost = [1 + int(h[p]) for p in ks if p < n]
        slots = np.zeros(lanes * chase)  # a lane steps its slots together: makespan over slots
        for c in cost:
            i = int(np.argmin(slots))
            slots[i] += c
        dyn[w] = slots.max()
    return lock.max(), dyn.max(), float(h.mean()), float((h > 0).mean())


if __name__ == "__main__":
    from hbam import synth
    import orc
    nrec = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    data, _ = synth.make_bam(nrec, as_numpy=False)
    s = orc.Stream(data)
    u = bytes(s.data)
    B = s.blocks
    tot = [0.0, 0.0]
    for k in range(1, 1 + nblk):
        a, n = int(B["ustart"][k]), int(B["isize"][k])
        raw = zlib.compressobj(5, zlib.DEFLATED, -15)
        c = raw.compress(u[a:a + n]) + raw.flush()
        toks = tokens(c)
        src = source_map(toks, n)
        d = depths(src)
        lit = float((src < 0).mean())
        l, y, hm, hf = simulate(src)
        tot[0] += l
        tot[1] += y
        print(f"block {k}: isize {n} tokens {len(toks)} literal positions {lit:.3f} mean depth {d.mean():.2f} "
              f"max {d.max()} | hops after compression mean {hm:.2f}, >0 {hf:.2f} | wave-steps (slowest wave): "
              f"lockstep {l:.0f} dynamic {y:.0f}", flush=True)
    print(f"mean lockstep {tot[0] / nblk:.0f} dynamic {tot[1] / nblk:.0f}")
