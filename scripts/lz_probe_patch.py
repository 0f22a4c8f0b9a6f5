#!/usr/bin/env python3
"""Development aid: per-step clock probes in k_inflate_lz77 (phase B).
`apply` saves the clean hbam_kernels.hip / hbam_pipeline.cpp / hbam_launch.h
under /tmp and writes probed copies (cycles per step summed over blocks,
printed by the pipeline after each inflate when HBAM_LZ_STATS is set);
`revert` restores them.  Build the probed library as a variant:
  python scripts/lz_probe_patch.py apply && (cd hadoop-bam_amd && make BUILD=build_lzp \\
    LIBOUT=lib/variants/libhbam_lzp.so) ; python scripts/lz_probe_patch.py revert"""
import shutil
import sys

K = "hadoop-bam_amd/csrc/hbam_kernels.hip"
PL = "hadoop-bam_amd/csrc/hbam_pipeline.cpp"
LH = "hadoop-bam_amd/csrc/hbam_launch.h"

KEDITS = [  # (anchor, text, insert after the anchor?)
    ("__global__ __launch_bounds__(kLzThreads) void k_inflate_lz77(",
     "__device__ unsigned long long g_lz_probe[8];\n"
     "#define LZP(k) do { if (threadIdx.x == 0) { const uint64_t t1_ = clock64(); "
     "atomicAdd(&g_lz_probe[k], (unsigned long long)(t1_ - lz_t0)); lz_t0 = t1_; } } while (0)\n", False),
    ("  const uint32_t nseg = (uint32_t)((gend - g0 + 15) >> 4);\n", "  uint64_t lz_t0 = clock64();\n", True),
    ("  const uint32_t whi = min(P + wsum, isize);  // end of this wave's range (the last token may run past ISIZE)\n",
     "  LZP(0);\n", True),
    ("  // 3. match bodies: every 0 entry belongs to the match whose distance is the", "  LZP(1);\n", False),
    ("  // 4. resolve, increasing positions first; results written back in place", "  LZP(2);\n", False),
    ("  // 5. 16 B stores; low bytes of 16 entries packed with v_perm", "  LZP(3);\n", False),
    ("        if (g >= blk.ustart && g < gend) u[g] = (uint8_t)map[16 * s + j];\n      }\n    }\n  }\n",
     "  LZP(4);\n", True),
    ("hipError_t launch_inflate_lz77(",
     "hipError_t lz_probe_read(unsigned long long* t) { return hipMemcpyFromSymbol(t, HIP_SYMBOL(g_lz_probe), 64); }\n",
     False),
]
PEDITS = [
    ("  float tab_ms = 0, huff_ms = 0, lz_ms = 0;",
     "  if (any && getenv(\"HBAM_LZ_STATS\")) {\n    unsigned long long t[8];\n    HIPCHK(hipStreamSynchronize(sB));\n"
     "    HIPCHK(lz_probe_read(t));\n    fprintf(stderr, \"[lz] Mcycles so far: tokens %.1f heads %.1f bodies %.1f resolve %.1f "
     "store %.1f\\n\", t[0] / 1e6, t[1] / 1e6, t[2] / 1e6, t[3] / 1e6, t[4] / 1e6);\n  }\n", False),
]
LEDITS = [("hipError_t launch_inflate_lz77(", "hipError_t lz_probe_read(unsigned long long* t);\n", False)]


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
