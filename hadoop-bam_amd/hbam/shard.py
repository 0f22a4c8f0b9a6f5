"""One BAM read by N processes / GPUs.

The reference parallelises the read path only by input splits: Hadoop cuts the
file into byte-range FileSplits, BAMInputFormat.addProbabilisticSplits
(BAMInputFormat.java:469-530) turns each into a FileVirtualSplit with
BAMSplitGuesser.guessNextBAMRecordStart (BAMSplitGuesser.java:108-235), merges
a split without a record start into the previous one (:497-513), and each
split is decoded independently by a BAMRecordReader.

ShardedBamReader does the same with one split per rank (torch.distributed, one
process per GPU):

  1. split r = bytes [r*S, (r+1)*S) of the file, S = ceil(size / world)
     (FileInputFormat with split size S);
  2. alignedBeg = guess(beg, end) on the rank's own device, alignedEnd =
     end<<16 | 0xffff (:490-495);
  3. all_gather of (alignedBeg, alignedEnd, empty): the empty-split merge of
     :497-513 applied to the gathered list (a split with no record start extends
     the previous one; an empty first split is the reference's IOException);
  4. each rank decodes its FileVirtualSplit (BAMRecordReader span rule);
  5. all_gather of the record counts -> global ordinals, and the
     .splitting-bai entries of each rank's records (ordinals k*g-1,
     SplittingBAMIndexer.java:262-287) gathered on rank 0, which prepends the
     first record's voff and appends size<<16.

The only collectives are the metadata all_gathers above (RCCL on GPUs, gloo in
the CPU tests); no record bytes cross ranks -- the reference's span rule already
assigns every record to exactly one split, and a rank reads the bytes of a
record that straddles its end from the file itself.  The index is built from
reader-decoded voffs, which equal the indexer's on a well-formed BAM.

`decoder` is any object with the hbam.BamFile interface used here
(guess_record_starts, decode_span, header / first_record_voff); the product
path passes hbam.BamFile, the CPU tests pass an adapter over the oracle.
"""
import numpy as np


def file_splits(size, world):
    """FileInputFormat byte ranges [(start, length)] for split size ceil(size/world)."""
    step = -(-size // world)
    out = []
    for r in range(world):
        a = min(size, r * step)
        b = min(size, (r + 1) * step)
        out.append((a, b - a))
    return out


def merge_empty_splits(aligned):
    """BAMInputFormat.java:497-513 over the gathered per-rank splits.

    aligned[r] = (alignedBeg, alignedEnd, empty).  Returns per rank the
    FileVirtualSplit (vStart, vEnd) it decodes, or None."""
    if not aligned or aligned[0][2]:
        raise IOError("no reads in first split: bad BAM file or tiny split size?")
    out = [None] * len(aligned)
    prev = None
    for r, (beg, end, empty) in enumerate(aligned):
        if empty:
            out[prev] = (out[prev][0], end)  # previousSplit.setEndVirtualOffset(alignedEnd)
        else:
            out[r] = (beg, end)
            prev = r
    return out


def be64(values):
    return b"".join(int(v).to_bytes(8, "big") for v in values)


class ShardedBamReader:
    def __init__(self, decoder, size, first_record_voff, rank, world, all_gather):
        """all_gather(obj) -> list of every rank's obj (torch.distributed.all_gather_object)."""
        self.dec = decoder
        self.size = size
        self.first_voff = first_record_voff
        self.rank = rank
        self.world = world
        self.all_gather = all_gather

    def split(self):
        beg, length = file_splits(self.size, self.world)[self.rank]
        end = beg + length
        if length == 0:
            mine = (end, (end << 16) | 0xFFFF, True)
        else:
            aligned_beg = int(self.dec.guess_record_starts([beg], [end])[0])
            mine = (aligned_beg, (end << 16) | 0xFFFF, aligned_beg == end)
        return merge_empty_splits(self.all_gather(mine))[self.rank]

    def run(self, granularity=4096):
        """Decode this rank's split; returns (records dict or None, global ordinal
        base, total records, .splitting-bai bytes on rank 0 else None)."""
        span = self.split()
        recs = self.dec.decode_span(*span) if span is not None else None
        n = 0 if recs is None else len(recs["voff"])
        counts = self.all_gather(n)
        base = sum(counts[:self.rank])
        total = sum(counts)
        ent = []
        if n and granularity > 0:
            o = np.arange(base, base + n, dtype=np.uint64)
            sel = ((o + 1) % np.uint64(granularity)) == 0
            ent = [int(v) for v in recs["voff"][sel]]
        gathered = self.all_gather(ent)
        sbi = None
        if self.rank == 0:
            allent = [e for part in gathered for e in part]
            sbi = be64([self.first_voff] + allent + [self.size << 16])
        return recs, base, total, sbi
