#!/usr/bin/env python3
"""Development aid: add (apply) or remove (revert) per-phase clock probes in
the inflate kernels of hbam_kernels.hip.  The product source never carries
them: `apply` saves the clean file to /tmp/hbam_kernels.clean.hip and writes
the probed one; `revert` restores it.  scripts/probe_inflate.py reads them
through hbam_probe_read."""
import shutil
import sys

P = "hadoop-bam_amd/csrc/hbam_kernels.hip"
SAVE = "/tmp/hbam_kernels.clean.hip"

EDITS = [
    ("namespace hbam {\n",
     "namespace hbam {\n__device__ unsigned long long g_prb[32];\n"
     "#define PRB_T() ((unsigned long long)clock64())\n"
     "#define PRB_ADD(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_prb[i], (unsigned long long)(v)); } while (0)\n"),
    ("  const uint32_t bi = b0 + blockIdx.x;\n  const BlockInfo blk = blocks[bi];\n  const uint32_t isize = blk.isize;",
     "  const uint32_t bi = b0 + blockIdx.x;\n  unsigned long long pt0 = PRB_T(), pt1;\n"
     "  const BlockInfo blk = blocks[bi];\n  const uint32_t isize = blk.isize;"),
    ("  __syncthreads();\n  // compressed bits: the LDS copy, or (unstaged) the file in HBM",
     "  __syncthreads();\n  pt1 = PRB_T(); PRB_ADD(0, pt1 - pt0); PRB_ADD(15, 1);\n"
     "  // compressed bits: the LDS copy, or (unstaged) the file in HBM"),
    ("  for (;;) {\n    if (wave == 0) {\n      uint32_t act = kActDone;",
     "  for (;;) {\n    unsigned long long ph0 = PRB_T();\n    if (wave == 0) {\n      uint32_t act = kActDone;"),
    ("    __syncthreads();\n    if (C.act != kActDecode) break;\n",
     "    __syncthreads();\n    unsigned long long ph1 = PRB_T(); PRB_ADD(1, ph1 - ph0);\n"
     "    if (C.act != kActDecode) break;\n    PRB_ADD(2, 1);\n"),
    ("    const uint32_t sx = x, snt = nt, snb = nb, sev = ev;\n",
     "    const uint32_t sx = x, snt = nt, snb = nb, sev = ev;\n"
     "    unsigned long long ph2 = PRB_T(); PRB_ADD(3, ph2 - ph1);\n"),
    ("    const uint32_t lend0 = wg_min(",
     "    unsigned long long ph3 = PRB_T(); PRB_ADD(4, ph3 - ph2);\n    const uint32_t lend0 = wg_min("),
    ("    uint32_t x3 = a, nt3 = 0, nb3 = 0, ev3 = EV_STOP;\n",
     "    uint32_t x3 = a, nt3 = 0, nb3 = 0, ev3 = EV_STOP;\n"
     "    unsigned long long ph4 = PRB_T(); PRB_ADD(5, ph4 - ph3);\n"),
    ("      C.m3any = m3 != 0xffffffffu;\n    }\n    __syncthreads();\n  }",
     "      C.m3any = m3 != 0xffffffffu;\n    }\n    __syncthreads();\n    PRB_ADD(6, PRB_T() - ph4);\n  }"),
    ("      hout[bi] = HuffOut{ntok, err, 0u, outpos};\n    }\n  }\n}",
     "      hout[bi] = HuffOut{ntok, err, 0u, outpos};\n    }\n  }\n  PRB_ADD(7, PRB_T() - pt0);\n}"),
    ("  const uint32_t nseg = (uint32_t)((gend - g0 + 15) >> 4);\n\n  if (isize > kMapMax) {",
     "  const uint32_t nseg = (uint32_t)((gend - g0 + 15) >> 4);\n  unsigned long long q0 = PRB_T();\n"
     "  PRB_ADD(16, 1);\n\n  if (isize > kMapMax) {"),
    ("  const uint32_t whi = min(P + wsum, isize);  // end of this wave's range (the last token may run past ISIZE)\n",
     "  const uint32_t whi = min(P + wsum, isize);  // end of this wave's range (the last token may run past ISIZE)\n"
     "  unsigned long long q1 = PRB_T(); PRB_ADD(17, q1 - q0);\n"),
    ("    for (uint32_t r = pos; r < hb; ++r, v += delta) m[r] = (uint16_t)v;\n  }\n  __syncthreads();\n",
     "    for (uint32_t r = pos; r < hb; ++r, v += delta) m[r] = (uint16_t)v;\n  }\n  __syncthreads();\n"
     "  unsigned long long q2 = PRB_T(); PRB_ADD(18, q2 - q1);\n"),
    ("    if (has2) m[q2] = (uint16_t)v2;\n  }\n  __syncthreads();\n",
     "    if (has2) m[q2] = (uint16_t)v2;\n  }\n  __syncthreads();\n"
     "  unsigned long long q3 = PRB_T(); PRB_ADD(19, q3 - q2);\n"),
    ("        if (g >= blk.ustart && g < gend) u[g] = (uint8_t)map[16 * s + j];\n      }\n    }\n  }\n}",
     "        if (g >= blk.ustart && g < gend) u[g] = (uint8_t)map[16 * s + j];\n      }\n    }\n  }\n"
     "  PRB_ADD(20, PRB_T() - q3);\n  PRB_ADD(21, PRB_T() - q0);\n}"),
    ("hipError_t launch_inflate_lz77(",
     'extern "C" int hbam_probe_read(unsigned long long* out, int reset) {\n'
     "  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prb), sizeof(unsigned long long) * 32) != hipSuccess) return 1;\n"
     "  if (reset) {\n    unsigned long long z[32] = {0};\n"
     "    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prb), z, sizeof z) != hipSuccess) return 2;\n  }\n  return 0;\n}\n"
     "hipError_t launch_inflate_lz77("),
]


def main():
    if sys.argv[1] == "apply":
        s = open(P).read()
        shutil.copy(P, SAVE)
        for a, b in EDITS:
            if s.count(a) != 1:
                raise SystemExit(f"anchor not unique/found: {a[:60]!r} ({s.count(a)})")
            s = s.replace(a, b)
        open(P, "w").write(s)
    else:
        shutil.copy(SAVE, P)


if __name__ == "__main__":
    main()
