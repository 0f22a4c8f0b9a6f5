"""Concurrent splits on one GPU (developer probe): the C2 file cut into K
FileVirtualSplits (FileInputFormat ranges + BAMSplitGuesser + the empty-split
merge, hbam/shard.py), each decoded by its own context (hbam_decode_span_device,
compressed bytes resident) from its own host thread, all K at once -- as K map
tasks sharing one GPU would.  Prints per K the aggregate inflated GB/s, the
record total (must equal the file's) and the per-split times.
--procs: the K splits decoded by K processes (K contexts of K processes,
each with its own hardware queues) instead of K threads of one process.
usage: python scripts/concurrent_probe.py [records] [K,K,...] [--procs]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hadoop-bam_amd"))
import hbam  # noqa: E402
from hbam import shard, synth  # noqa: E402


def run(path, size, u, n_rec, k, reps=5):
    fs = [hbam.BamFile(path=path) for _ in range(k)]
    try:
        first = fs[0].header()["first_record_voff"]
        aligned = []
        for beg, length in shard.file_splits(size, k):
            end = beg + length
            g = int(fs[0].guess_record_starts([beg], [end])[0]) if length else end
            aligned.append((g, (end << 16) | 0xFFFF, g == end))
        spans = shard.merge_empty_splits(aligned)
        work = [(f, s) for f, s in zip(fs, spans) if s is not None]
        for f, (vs, ve) in work:
            f.prefetch(vs >> 16, min(size, (ve >> 16) + (256 << 10)))
        recs = [0] * len(work)
        times = [0.0] * len(work)

        def one(i):
            f, (vs, ve) = work[i]
            t = time.perf_counter()
            recs[i] = f.decode_span_device(vs, ve, digest=False)["records"]
            times[i] = time.perf_counter() - t

        def step():
            th = [threading.Thread(target=one, args=(i,)) for i in range(len(work))]
            for t in th:
                t.start()
            for t in th:
                t.join()

        step()
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            step()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        assert sum(recs) == n_rec, (sum(recs), n_rec)
        print(f"K={k}: {best * 1e3:.3f} ms  {u / best / 1e9:.1f} GB/s U  records {sum(recs)}  "
              f"split ms {[round(x * 1e3, 2) for x in times]}", flush=True)
    finally:
        for f in fs:
            f.close()


def proc_worker(path, span, size, bar, q, reps):
    f = hbam.BamFile(path=path)
    try:
        vs, ve = span
        f.prefetch(vs >> 16, min(size, (ve >> 16) + (256 << 10)))
        f.decode_span_device(vs, ve, digest=False)
        ts, n = [], 0
        for _ in range(reps):
            bar.wait(timeout=60)
            t = time.perf_counter()
            n = f.decode_span_device(vs, ve, digest=False)["records"]
            ts.append(time.perf_counter() - t)
            bar.wait(timeout=60)
        q.put((n, ts))
    finally:
        f.close()


def run_procs(path, size, u, n_rec, k, reps=5):
    import multiprocessing as mp
    f0 = hbam.BamFile(path=path)
    try:
        aligned = []
        for beg, length in shard.file_splits(size, k):
            end = beg + length
            g = int(f0.guess_record_starts([beg], [end])[0]) if length else end
            aligned.append((g, (end << 16) | 0xFFFF, g == end))
        spans = [s_ for s_ in shard.merge_empty_splits(aligned) if s_ is not None]
    finally:
        f0.close()
    ctx = mp.get_context("spawn")
    bar = ctx.Barrier(len(spans))
    q = ctx.Queue()
    ps = [ctx.Process(target=proc_worker, args=(path, sp, size, bar, q, reps), daemon=True) for sp in spans]
    for p_ in ps:
        p_.start()
    res = [q.get(timeout=120) for _ in ps]
    for p_ in ps:
        p_.join(timeout=60)
    assert sum(r[0] for r in res) == n_rec, (sum(r[0] for r in res), n_rec)
    rep = [max(r[1][i] for r in res) for i in range(reps)]
    best = min(rep)
    print(f"K={k} processes: {best * 1e3:.3f} ms  {u / best / 1e9:.1f} GB/s U  records {n_rec}", flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else n
    ks = [int(x) for x in args[1].split(",")] if len(args) > 1 else [1, 2, 3, 4]
    data, info = synth.make_bam(n, as_numpy=True)
    path = "/dev/shm/hbam_concurrent_probe.bam"
    data.tofile(path)
    del data
    try:
        for k in ks:
            if "--procs" in sys.argv:
                run_procs(path, info["compressed"], info["uncompressed"], n, k)
            else:
                run(path, info["compressed"], info["uncompressed"], n, k)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
