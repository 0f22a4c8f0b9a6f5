"""Coordinate-sorted BAMs for the BAI split calculator tests: synthetic reads
moved onto several contigs (with empty contigs between them) by rewriting
refID / pos / bin / mate fields of a generated BAM, recompressed with the
original block cuts.  Test data only."""
import struct

import bai
import orc
from hbam import synth
from test_gpu_windows import recompress


def spread_bam(n_records, placement, seed=0x48424D00, block_payload=65280):
    """placement = [(refID, first_pos, step)]: the records are dealt to the
    contigs in order, consecutive positions `step` apart."""
    data, _ = synth.make_bam(n_records, seed=seed, block_payload=block_payload)
    s = orc.Stream(data, stringency=orc.SILENT)
    rc, r = s.decode_all()
    assert rc == 0
    u = bytearray(s.data)
    n = len(r["offset"])
    per = -(-n // len(placement))
    for i, p in enumerate(r["offset"]):
        p = int(p)
        ref, first, step = placement[min(i // per, len(placement) - 1)]
        pos = first + (i % per) * step
        _, _, end, flag = bai._ref_span(u, p)
        span = end - struct.unpack_from("<i", u, p + 8)[0]
        struct.pack_into("<ii", u, p + 4, ref, pos)
        if flag & 4:
            b = bai._reg2bin(pos, pos + 1)
        else:
            b = bai._reg2bin(pos, pos + span)
        struct.pack_into("<H", u, p + 14, b)
        if flag & 1:  # mate on the same contig, nearby
            struct.pack_into("<ii", u, p + 24, ref, pos + 200)
    return recompress(s, bytes(u))
