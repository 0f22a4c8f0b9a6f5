#!/usr/bin/env python3
"""Benchmark of the MI355X BAM read hot path (BASELINE.json metric).

One "step" = one full pass of the hot path over one synthetic BAM resident in
HBM: BGZF block discovery -> inflate (Huffman phase + LZ77 phase) -> record
boundary scan -> fused field decode + sort keys + voffs.  Workload: config C2,
a synthetic 10M x 150 bp paired-end coordinate-sorted BAM (generated on the
box, zlib level 5 as htsjdk writes).  With N GPUs each rank owns one C2-sized
BGZF shard (weak scaling; shards are independent, no data-path collective).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "uncompressed BAM decode GB/s + records/sec per GPU and 8-GPU node"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(data, info, seconds):
    """Oracle (zlib inflate + htsjdk-rule record chain + keys) on the host, one
    thread, on a prefix of the same BAM sized to ~`seconds` of work."""
    import orc
    import numpy as np
    # calibrate on a small prefix (whole BGZF blocks), then scale up
    blocks = []
    p = 0
    while p < len(data):
        bs = int.from_bytes(data[p + 16:p + 18], "little") + 1
        blocks.append((p, bs))
        p += bs
    def run(nb):
        end = blocks[nb - 1][0] + blocks[nb - 1][1]
        t = time.perf_counter()
        s = orc.Stream(data[:end])
        rc, r = s.decode_span(s.first_record_voff, (1 << 64) - 1)
        dt = time.perf_counter() - t
        return dt, s.data_len, len(r["key"])
    nb = min(len(blocks), 200)
    dt, u, n = run(nb)
    target = max(nb, min(len(blocks), int(nb * seconds / max(dt, 1e-3))))
    dt, u, n = run(target)
    return {"value": round(u / dt / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "records_per_s": round(n / dt, 1),
            "sample": f"first {target} BGZF blocks ({u} inflated bytes, {n} records) of the same C2 BAM, "
                      f"oracle/hbam_oracle.c (system zlib) single thread, {dt:.1f} s"}


def extra_configs(c2, c2_info):
    """Side measurements reported next to the headline (not part of `value`):
    C5-style .splitting-bai generation (g=4096) over the same C2 BAM through
    the SplittingBAMIndexer entry point (hbam_build_splitting_index: inflate +
    indexer-rule chain + entry emit, file resident in HBM), and a C4-like
    long-read BAM (ONT-style 10-50 kb reads, records spanning blocks) through
    the same device pipeline as the headline."""
    import hbam
    from hbam import synth
    res = {}
    f = hbam.BamFile(c2.tobytes() if hasattr(c2, "tobytes") else c2)
    t = time.perf_counter()
    sbi = f.splitting_index(4096)
    dt = time.perf_counter() - t
    res["c5_splitting_bai_g4096_on_c2"] = {
        "entries": len(sbi) // 8, "seconds": round(dt, 4),
        "uncompressed_GBps": round(c2_info["uncompressed"] / dt / 1e9, 3),
        "note": "first call: includes inflating every block (resident compressed file)"}
    f.close()
    data, info = synth.make_bam(12000, mode="long", as_numpy=True, seed=0x48424D04)
    g = hbam.Gpu(0)
    g.load(data)
    g.run(timing=True)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        st = g.run(timing=True)
        ts.append(time.perf_counter() - t)
    dt = min(ts)
    res["c4_long_reads"] = {
        "records": int(st["records"]), "compressed_bytes": info["compressed"],
        "uncompressed_bytes": info["uncompressed"], "seconds": round(dt, 5),
        "uncompressed_GBps": round(info["uncompressed"] / dt / 1e9, 3),
        "stages_ms": {k: round(st[k], 3) for k in ("ms_locate", "ms_huff", "ms_lz77", "ms_chain", "ms_decode")}}
    g.close()
    return res


def host_and_copy_legs(g, data, info, pass_ms):
    """Measurements around the headline (rank 0, N=1; never `value`):
    * SAMRecordWritable.write of the whole decoded C2 span on the GPU
      (k_wr_copy + k_wr_bin_patch; 2 B of HBM traffic per encoded byte);
    * the PCIe-inclusive rate: the compressed file copied host->HBM from
      pinned memory (hbam_gpu_reload, HIP events) plus one device pass,
      serial, the bound if the copy were fully overlapped, and the measured
      overlapped pass (hbam_gpu_run_streamed: pieces copied on a copy stream
      while landed pieces are located + inflated), checked equal to the
      device-resident results;
    * measured hipMemcpy device-to-device bandwidth (2 B per byte),
      the practical ceiling the HBM-bound kernels are compared with."""
    res = {}
    ms, nb = g.encode_writables(iters=10)
    res["writable_encode"] = {
        "bytes": nb, "ms": round(ms, 4), "GBps_encoded": round(nb / ms / 1e6, 2),
        "roofline": {"bound": "hbm", "achieved": round(2 * nb / ms / 1e6, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(2 * nb / ms / 1e6 / HBM_PEAK_GBS, 4)}}
    h2d = min(g.reload(data.ctypes.data, data.nbytes, pinned=True) for _ in range(3))
    pageable = g.reload(data.ctypes.data, data.nbytes, pinned=False)
    res["pcie_inclusive"] = {
        "h2d_ms_pinned": round(h2d, 3), "h2d_GBps_pinned": round(data.nbytes / h2d / 1e6, 2),
        "h2d_ms_pageable": round(pageable, 3), "pass_ms": round(pass_ms, 3),
        "serial_uncompressed_GBps": round(info["uncompressed"] / (h2d + pass_ms) / 1e6, 2),
        "overlapped_bound_uncompressed_GBps": round(info["uncompressed"] / max(h2d, pass_ms) / 1e6, 2)}
    # copy overlapped with locate + inflate of the pieces already in HBM
    import hbam
    import numpy as np
    k_ref, v_ref = g.fetch(int(info["n_records"]))
    with hbam.PinnedBuffer(data.nbytes) as pb:
        pb.array[:] = data
        best = {}
        for piece in (32 << 20, 64 << 20):
            ts = []
            for _ in range(3):
                st = g.run_streamed(pb.ptr, data.nbytes, piece)
                ts.append(st["ms_total"])
            best[piece] = min(ts)
        k_s, v_s = g.fetch(int(info["n_records"]))
    piece, ms_s = min(best.items(), key=lambda kv: kv[1])
    res["pcie_inclusive"].update({
        "streamed_ms": round(ms_s, 3), "streamed_piece_bytes": piece,
        "streamed_uncompressed_GBps": round(info["uncompressed"] / ms_s / 1e6, 2),
        "streamed_records_per_s": round(info["n_records"] / ms_s * 1e3, 1),
        "streamed_matches_resident": bool(np.array_equal(k_s, k_ref) and np.array_equal(v_s, v_ref))})
    res["bgzf_write"] = bgzf_write_leg(g, data, info)
    d2d = g.d2d_bandwidth(1 << 32, 5)
    res["d2d_copy_GBps_measured"] = round(d2d, 1)
    res["writable_encode"]["frac_of_measured_d2d"] = round(2 * nb / ms / 1e6 / d2d, 4)
    return res


def bgzf_write_leg(g, data, info):
    """BGZF write path: the resident inflated C2 stream
    recompressed on the GPU with the file's block boundaries at zlib level 5
    (hbam_gpu_bgzf_compress: k_deflate_blocks + k_dfl_crc + k_dfl_frame),
    checked byte-identical to the generated file; the CPU leg is the oracle
    (system zlib, htsjdk's deflater lifecycle) on the first 200 blocks."""
    import zlib
    import numpy as np
    import orc
    g.bgzf_compress(level=5, eof=False, iters=0)  # allocation + warm-up
    ms, nb = g.bgzf_compress(level=5, eof=False, iters=1)
    same = nb == data.nbytes and bool(np.array_equal(g.fetch_compressed(0, nb), data))
    u, c = info["uncompressed"], info["compressed"]
    raw = data[:min(data.nbytes, 200 * 65536 * 2)].tobytes()
    p, pay, lens = 0, [], []
    while len(lens) < 200 and p + 18 <= len(raw):
        bs = int.from_bytes(raw[p + 16:p + 18], "little") + 1
        if p + bs > len(raw):
            break
        x = zlib.decompressobj(-15).decompress(raw[p + 18:p + bs - 8])
        pay.append(x)
        lens.append(len(x))
        p += bs
    sample = b"".join(pay)
    t = time.perf_counter()
    orc.bgzf_compress(sample, lens, level=5, eof=False)
    dt = time.perf_counter() - t
    return {"level": 5, "ms": round(ms, 2), "uncompressed_GBps": round(u / ms / 1e6, 4),
            "identical_to_file": same, "bytes_out": int(nb),
            "roofline": {"bound": "latency (serial LZ77 recurrence per block)", "achieved": round((u + c) / ms / 1e6, 4),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round((u + c) / ms / 1e6 / HBM_PEAK_GBS, 7)},
            "cpu_baseline": {"value": round(len(sample) / dt / 1e9, 5), "unit": "GB/s", "cores": 1, "kind": "port",
                             "sample": f"first {len(lens)} blocks ({len(sample)} B) through oracle orc_bgzf_compress "
                                       f"(system zlib 1.2.11, level 5), {dt:.2f} s"}}


def pmc_traffic(kernels):
    """HBM bytes per launch of `kernels` (summed) from the newest committed
    rocprofv3 PMC summary (profiles/*/summary.json, written by
    profiles/collect.sh + summarize.py: FETCH_SIZE x1024 x2 gfx950 correction,
    WRITE_SIZE x1024).  None when no summary is committed."""
    import glob
    best = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "summary.json")))
    if not best:
        return None, None
    try:
        ks = json.load(open(best[-1]))["kernels"]
        tot = 0.0
        for k in kernels:  # phase A is templated on LDS staging: C2 runs the staged instance
            e = ks[k] if k in ks else ks[k + "<true>"]
            tot += e["main_fetch_bytes_corrected"] + e["main_write_bytes"]
        return int(tot), os.path.relpath(best[-1], ROOT)
    except (KeyError, ValueError, OSError):
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-bam", default=None)
    ap.add_argument("--no-extra", action="store_true", help="skip the C4 / index side measurements (the io legs always run at N=1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    import numpy as np
    import hbam
    from hbam import synth

    t0 = time.time()
    data, info = synth.make_bam(args.records, seed=0x48424D00 + 7919 * rank, as_numpy=True)
    log(f"[rank {rank}] generated C2 shard: {info} in {time.time() - t0:.1f}s")
    if args.save_bam and rank == 0:
        data.tofile(args.save_bam)

    g = hbam.Gpu(local_rank)
    g.load(data)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        st = g.run(timing=True)
    barrier()
    stats = []
    t = time.perf_counter()
    for _ in range(args.steps):
        stats.append(g.run(timing=True))
    barrier()
    elapsed = time.perf_counter() - t
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tot = torch.tensor([float(info["uncompressed"]), float(stats[-1]["records"]), float(info["compressed"])],
                           dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tot)
        u_all, n_all, c_all = (float(x) for x in tot.tolist())
    else:
        u_all, n_all, c_all = float(info["uncompressed"]), float(stats[-1]["records"]), float(info["compressed"])

    st = stats[-1]
    assert st["records"] == args.records, (st["records"], args.records)
    ms_step = elapsed / args.steps * 1e3
    value = u_all * args.steps / elapsed / 1e9

    # dominant kernel pair: inflate (phase A huff + phase B lz77), launched as
    # pairs over chunks of BGZF blocks; HIP events on the pipeline stream.
    n_launch = max(1, st["inflate_launches"])
    infl_ms = sum(s_["ms_huff"] + s_["ms_lz77"] for s_ in stats) / len(stats) / n_launch
    huff_ms = sum(s_["ms_huff"] for s_ in stats) / len(stats) / n_launch
    lz_ms = sum(s_["ms_lz77"] for s_ in stats) / len(stats) / n_launch
    alg_bytes = (info["compressed"] + info["uncompressed"]) / n_launch  # C read + U written per launch pair
    achieved = alg_bytes / (infl_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(("hbam::k_inflate_huff", "hbam::k_inflate_lz77"))
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (tools/gen_synth_bam.c, zlib level 5 BGZF, generated on the box)",
        "config": {"workload": "C2: synthetic 10M x 150bp paired-end coordinate-sorted BAM per GPU",
                   "records_per_gpu": args.records, "compressed_bytes_per_gpu": info["compressed"],
                   "uncompressed_bytes_per_gpu": info["uncompressed"], "bgzf_blocks_per_gpu": info["blocks"],
                   "parallelism": f"bgzf-shard x{world}"},
        "records_per_s": round(n_all * args.steps / elapsed, 1),
        "link_fallbacks": int(sum(s_["link_fallbacks"] for s_ in stats)),
        "link_rewalks": int(sum(s_["link_rewalks"] for s_ in stats)),
        "stages_ms": {k: round(st[k], 3) for k in ("ms_locate", "ms_inflate", "ms_huff", "ms_lz77", "ms_chain",
                                                    "ms_decode", "ms_total")},
        "roofline": {"bound": "hbm", "kernel": "k_inflate_huff+k_inflate_lz77 (one launch pair)",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "launches_per_pass": n_launch, "avg_launch_ms": round(infl_ms, 3),
                     "huff_avg_launch_ms": round(huff_ms, 3), "lz77_avg_launch_ms": round(lz_ms, 3),
                     "alg_bytes_per_launch": int(alg_bytes)},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1:
        out["io"] = host_and_copy_legs(g, data, info, ms_step)
    if rank == 0 and world == 1 and not args.no_extra:
        g.close()
        out["extra"] = extra_configs(data, info)
    if rank == 0 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(data.tobytes(), info, args.cpu_seconds)
        except Exception as e:  # reported, never substituted for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
