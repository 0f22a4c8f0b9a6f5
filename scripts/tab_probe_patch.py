#!/usr/bin/env python3
"""Development aid: per-step clock probes in k_huff_tables (the phase-A
header parse + table build).  `apply` saves the clean hbam_kernels.hip /
hbam_pipeline.cpp / hbam_launch.h under /tmp and writes probed copies (cycles
per step summed over headers, printed by the pipeline after each inflate when
HBAM_TAB_STATS is set); `revert` restores them.  Build as a variant:
  python scripts/tab_probe_patch.py apply && (cd hadoop-bam_amd && make BUILD=build_tabp \\
    LIBOUT=lib/variants/libhbam_tabp.so) ; python scripts/tab_probe_patch.py revert"""
import shutil
import sys

K = "hadoop-bam_amd/csrc/hbam_kernels.hip"
PL = "hadoop-bam_amd/csrc/hbam_pipeline.cpp"
LH = "hadoop-bam_amd/csrc/hbam_launch.h"

KEDITS = [  # (anchor, text, insert after the anchor?)
    ("template <bool REG>\n__device__ int dyn_header_par(",
     "__device__ unsigned long long g_tab_probe[16];\n"
     "#define TBP(k) do { if (lane_id() == 0 && (blockIdx.x & 63) == 0) { const uint64_t t1_ = clock64(); "
     "atomicAdd(&g_tab_probe[k], (unsigned long long)(t1_ - tb_t0)); tb_t0 = t1_; } } while (0)\n", False),
    ("  if (p + 14 > E) return DH_TRUNC;\n  const uint32_t h = rfl(peek32(W, p));\n",
     "  uint64_t tb_t0 = clock64();\n", False),
    ("  if (rfl(build_tab<REG>(L, L.cl_lens, 19, 7, 2, L.dist, L.cnt_dist, L.sort_dist, nullptr, 0))) return DH_TRUNC;\n",
     "  if constexpr (REG) TBP(1);\n", True),
    ("      // exit offset (from the slice start) when the decode enters at j; the\n", "      TBP(10);\n", False),
    ("      // entry of slice l = F_{l-1}(0), F_l = g_l o ... o g_0: an inclusive\n", "      TBP(11);\n", False),
    ("      // walk the true symbols from the entry, compacting them to ent[lane][0..ns)\n", "      TBP(14);\n", False),
    ("    // run lengths of this lane's symbols and its last defined value\n", "    if constexpr (REG) TBP(15);\n", False),
    ("    // write this lane's runs\n", "    if constexpr (REG) TBP(12);\n", False),
    ("    if (__ballot(bad)) return DH_TRUNC;\n    if (reach) {", "    if constexpr (REG) TBP(13);\n", False),
    ("  wave_sync();\n  if (rfl(L.lens[256]) == 0) return DH_TRUNC;\n", "  if constexpr (REG) TBP(2);\n", True),
    ("  if (rfl(build_tab<REG>(L, L.lens + hlit, (int)hdist, kDistRoot, 1, L.dist, L.cnt_dist, L.sort_dist, L.distsub,\n",
     "  if constexpr (REG) TBP(3);\n", False),
    ("                      kDistSubCap)))\n    return DH_TRUNC;\n", "  if constexpr (REG) TBP(4);\n", True),
    ("  if constexpr (REG) TBP(4);\n  pair_literals(L);\n", "  if constexpr (REG) TBP(5);\n", True),
    ("  const BlockInfo blk = blocks[bi];\n  HuffTableInfo ti{1u, 0u, 0u, 0u};\n", "  uint64_t tb_t0 = clock64();\n", True),
    ("    for (uint32_t i = lane; i <= nreal; i += 64) s_in[i] = src[i];  // +1 pad chunk (file is padded)\n    wave_sync();\n",
     "    TBP(0);\n", True),
    ("      if (dyn_header_par<true>(L, C, R.W, hp, E, &b0pos) == DH_OK) {\n        wave_sync();\n",
     "        tb_t0 = clock64();\n", True),
    ("        const uint32_t est = block_bits_estimate(L.lens, (h & 31) + 257, ((h >> 5) & 31) + 1);\n",
     "        TBP(6);\n", True),
    ("        ti = HuffTableInfo{0u, b0pos + 8u * sb, fin, est};\n",
     "        TBP(7);\n        wave_sync();\n        TBP(9);\n        if (lane == 0 && (blockIdx.x & 63) == 0) atomicAdd(&g_tab_probe[8], 1ull);\n", True),
    ("hipError_t launch_inflate_lz77(",
     "hipError_t tab_probe_read(unsigned long long* t) { return hipMemcpyFromSymbol(t, HIP_SYMBOL(g_tab_probe), 128); }\n",
     False),
]
PEDITS = [
    ("  float tab_ms = 0, huff_ms = 0, lz_ms = 0;",
     "  if (any && getenv(\"HBAM_TAB_STATS\")) {\n    unsigned long long t[16];\n    HIPCHK(hipDeviceSynchronize());\n"
     "    HIPCHK(tab_probe_read(t));\n    const double n = t[8] ? (double)t[8] : 1.0;\n"
     "    fprintf(stderr, \"[tab] headers %llu, cycles per header: stage %.0f cl %.0f lens %.0f lit %.0f dist %.0f "
     "pair %.0f est %.0f write %.0f probe %.0f (1 block in 64); lens: lookups %.0f backward %.0f runs+scans %.0f write %.0f chain %.0f walk %.0f\\n\", t[8], t[0] / n, t[1] / n, t[2] / n, t[3] / n, t[4] / n, t[5] / n, t[6] / n, t[7] / n, t[9] / n, t[10] / n, t[11] / n, t[12] / n, t[13] / n, t[14] / n, t[15] / n);\n  }\n", False),
]
LEDITS = [("hipError_t launch_inflate_lz77(", "hipError_t tab_probe_read(unsigned long long* t);\n", False)]


def edit(path, edits):
    s = open(path).read()
    shutil.copy(path, "/tmp/" + path.split("/")[-1] + ".clean")
    for a, b, after in edits:
        if s.count(a) != 1:
            raise SystemExit(f"{path}: anchor not unique/found: {a[:60]!r} ({s.count(a)})")
        s = s.replace(a, a + b if after else b + a)
    open(path, "w").write(s)


def main():
    if sys.argv[1] == "apply":
        edit(K, KEDITS)
        edit(PL, PEDITS)
        edit(LH, LEDITS)
    else:
        for p in (K, PL, LH):
            shutil.copy("/tmp/" + p.split("/")[-1] + ".clean", p)


if __name__ == "__main__":
    main()
