#!/usr/bin/env python3
"""Development aid (experiment build): HBAM_EXP_SKIPB=1 at run time makes the
phase-A emit walk store its tokens to one fixed 16 B slot per lane (lanes of
a wave contiguous: the stores coalesce) and skips phase B, so a timing pass
that follows one normal pass measures phase A with coalesced instead of
scattered token stores (the inflated bytes of the normal pass stay valid).
apply / revert like scripts/lz_probe_patch.py."""
import shutil
import sys

K = "hadoop-bam_amd/csrc/hbam_kernels.hip"
PL = "hadoop-bam_amd/csrc/hbam_pipeline.cpp"
LH = "hadoop-bam_amd/csrc/hbam_launch.h"
KE = [
    ("                                                uint32_t out0, uint32_t isize) {\n  constexpr bool EMIT = MODE == LD_EMIT;",
     "                                                uint32_t out0, uint32_t isize, bool fixed_slot = false) {\n"
     "  constexpr bool EMIT = MODE == LD_EMIT;"),
    ("        *reinterpret_cast<Tok4*>(tok + nt - 3) = Tok4{q0, q1, q2, q3};                      \\",
     "        *reinterpret_cast<Tok4*>(fixed_slot ? tok : tok + nt - 3) = Tok4{q0, q1, q2, q3};   \\"),
    ("        if (fs == 3) *reinterpret_cast<Tok4*>(tok + nt - 3) = Tok4{q0, q1, q2, q3};",
     "        if (fs == 3) *reinterpret_cast<Tok4*>(fixed_slot ? tok : tok + nt - 3) = Tok4{q0, q1, q2, q3};"),
    ("    uint32_t* p = tok + nt - fill;", "    uint32_t* p = fixed_slot ? tok : tok + nt - fill;"),
    ("      ev3 = lane_decode<LD_EMIT>(L, W, a, stop, E, x3, nt3, nb3, mp, mj, tok_out + tok0 + toff, out0 + boff, isize);",
     "      ev3 = lane_decode<LD_EMIT>(L, W, a, stop, E, x3, nt3, nb3, mp, mj,\n"
     "                                 defer >= 2 ? tokens + 4 * tid : tok_out + tok0 + toff, out0 + boff, isize,\n"
     "                                 defer >= 2);"),
    ("    if (defer) {  // the next header is the next round's (k_huff_tables)",
     "    if (defer & 1) {  // the next header is the next round's (k_huff_tables)"),
]
PE = [
    ("                                          tables_[par].p, tinfo_[par].p, r, r + 1 < kInflateRounds ? 1u : 0u,",
     "                                          tables_[par].p, tinfo_[par].p, r,\n"
     "                                          (r + 1 < kInflateRounds ? 1u : 0u) | (getenv(\"HBAM_EXP_SKIPB\") ? 2u : 0u),"),
    ("    HIPCHK(launch_inflate_lz77(dblocks_.p, cb, ce - cb, cu, tokens_[par].p, hout_.p, du_.p, sB));",
     "    if (!getenv(\"HBAM_EXP_SKIPB\"))\n"
     "      HIPCHK(launch_inflate_lz77(dblocks_.p, cb, ce - cb, cu, tokens_[par].p, hout_.p, du_.p, sB));"),
]


def edit(path, edits):
    s = open(path).read()
    shutil.copy(path, "/tmp/" + path.split("/")[-1] + ".clean")
    for a, b in edits:
        if s.count(a) != 1:
            raise SystemExit(f"{path}: anchor not unique/found: {a[:70]!r} ({s.count(a)})")
        s = s.replace(a, b)
    open(path, "w").write(s)


if __name__ == "__main__":
    if sys.argv[1] == "apply":
        edit(K, KE)
        edit(PL, PE)
    else:
        for p in (K, PL):
            shutil.copy("/tmp/" + p.split("/")[-1] + ".clean", p)
