#!/usr/bin/env python3
"""Benchmark of the MI355X BAM read hot path (BASELINE.json metric).

One "step" = one pass of the hot path over a rank's FileVirtualSplit of ONE
synthetic BAM, its compressed bytes already resident in HBM: BGZF block
discovery -> inflate (Huffman phase + LZ77 phase) -> record-boundary chain ->
fused field decode + sort keys + voffs into SoA columns in HBM
(hbam_decode_span_device, the BAMRecordReader path).

Workloads (config.workload):
  c2  (default at --gpus 1): BASELINE config 2, synthetic 10M x 150 bp
      paired-end (~1.4 GB compressed).  With N ranks: N x C2 records in one
      file, one split per rank (weak scaling) -- the side leg of an N>1 run.
  c3  (default at --gpus N>1): BASELINE config 3, ONE ~60 GB BAM split by
      BGZF byte ranges across the N ranks exactly as Hadoop-BAM plans it
      (FileInputFormat ranges -> BAMSplitGuesser -> empty-split merge,
      hbam/shard.py): strong scaling, total work fixed.  The same run gathers
      every rank's .splitting-bai entries at g = 4096 on rank 0 (config 5,
      SURVEY 8e) and checks them and an order-sensitive decode digest against
      the oracle run over the whole file on the host's cores.

Multi-rank runs write the file together (each rank generates its segments),
and each rank copies only its split's bytes to its GPU; the only collectives
are metadata all_gathers and the max-over-ranks timing all_reduce.

Prints ONE JSON line (rank 0).  Side legs at N=1 (rank 0): CPU baseline (the
oracle at 1 thread and on every usable host core), in-session PMC traffic of
the dominant kernel (rocprofv3 child runs), the drop-in call end to end
(hbam_open -> hbam_decode_span batches -> pinned host columns), C3 / C5 at
60 GB, C4 long reads, write-path legs.
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hadoop-bam_amd"))
# GPU_MAX_HW_QUEUES is left as the box sets it (4): libhbam's stream priority
# levels keep its decode, batch and staging streams on separate queues at 4
# (DESIGN.md 3), and the line records the value it ran at.

METRIC = "uncompressed BAM decode GB/s + records/sec per GPU and 8-GPU node"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
SEED = 0x48424D00
ALL = (1 << 64) - 1
BOUND_MIN = 0.7  # a limit below this is not called the bound (roofline.bound = "latency")
SOA_BYTES_PER_RECORD = 37  # key 8 + voff 8 + rest_off 8 + refID 4 + pos 4 + flag 2 + bin 2 + mapq 1
INFLATE_ROUNDS = 2  # hbam_device.h kInflateRounds: k_huff_tables + k_inflate_huff launches per chunk (tests/test_bench_launch.py)
BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """CPUs this process may use: the affinity set, capped by a cgroup quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def scratch_dir():
    return "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else tempfile.gettempdir()


def pwrite_all(fd, arr, off):
    mv = memoryview(arr).cast("B")
    done = 0
    while done < len(mv):
        done += os.pwrite(fd, mv[done:], off + done)


# ---------------------------------------------------------------------------
# the file
# ---------------------------------------------------------------------------
def build_shared_bam(path, rank, world, records, all_gather, barrier):
    """Each rank writes its segment of one BAM; returns (size, inflated bytes)."""
    from hbam import synth
    t = time.time()
    seg, info = synth.make_bam_segment(world * records, rank * records, (rank + 1) * records,
                                       with_header=rank == 0, eof_block=rank == world - 1, seed=SEED)
    sizes = all_gather((int(seg.nbytes), int(info["uncompressed"])))
    off = sum(s for s, _ in sizes[:rank])
    size = sum(s for s, _ in sizes)
    if rank == 0:
        with open(path, "wb") as fh:
            fh.truncate(size)
    barrier()
    fd = os.open(path, os.O_WRONLY)
    try:
        pwrite_all(fd, seg, off)
    finally:
        os.close(fd)
    barrier()
    log(f"[rank {rank}] wrote segment {seg.nbytes} B at {off} of {size} ({time.time() - t:.1f}s)")
    return size, sum(u for _, u in sizes)


# ---------------------------------------------------------------------------
# CPU baseline: the oracle (oracle/orc_scan.c) on the host's own cores
# ---------------------------------------------------------------------------
def cpu_baseline(path, size, seconds):
    """The restated read path (zlib inflate + htsjdk record rules + keys) on
    the host: all usable cores over the whole file (blocks cut into ranges,
    one per thread) and one thread over a prefix sized to ~`seconds`.
    Also returns the oracle's whole-file digest for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import orc
    data = np.memmap(path, np.uint8, mode="r", shape=(size,))
    cores = host_cores()
    t = time.perf_counter()
    full, _ = orc.scan(data, threads=cores, mode="decode")
    dt_all = time.perf_counter() - t
    if full["rc"] != 0:
        raise RuntimeError(f"oracle scan failed: {full}")
    # one thread: calibrate on 200 blocks, then ~`seconds` worth
    t = time.perf_counter()
    r1, _ = orc.scan(data, threads=1, mode="decode", max_blocks=200)
    dt = time.perf_counter() - t
    nb = max(200, min(int(full["blocks"]), int(200 * seconds / max(dt, 1e-3))))
    t = time.perf_counter()
    r1, _ = orc.scan(data, threads=1, mode="decode", max_blocks=nb)
    dt1 = time.perf_counter() - t
    model = cpu_model()
    out = {"value": round(full["u_bytes"] / dt_all / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
           "host_cores_total": os.cpu_count(), "cores_note": "cores = the threads used: every CPU the process may "
           "use (affinity set capped by the cgroup quota); host_cores_total = the machine's logical CPUs",
           "records_per_s": round(full["records"] / dt_all, 1), "cpu_model": model,
           "sample": f"whole file ({full['u_bytes']} inflated bytes, {full['records']} records) through "
                     f"oracle/orc_scan.c (system zlib, htsjdk reader rules, STRICT) on {cores} threads "
                     f"({model}), {dt_all:.2f} s",
           "single_thread": {"value": round(r1["u_bytes"] / dt1 / 1e9, 4), "unit": "GB/s", "cores": 1,
                             "records_per_s": round(r1["records"] / dt1, 1),
                             "sample": f"first {nb} BGZF blocks ({r1['u_bytes']} inflated bytes, "
                                       f"{r1['records']} records), 1 thread, {dt1:.1f} s"}}
    return out, full


# ---------------------------------------------------------------------------
# in-session PMC traffic of the dominant kernel (rocprofv3 child processes)
# ---------------------------------------------------------------------------
def pmc_child(path, vstart, vend):
    import hbam
    with hbam.BamFile(path=path) as f:
        f.prefetch(vstart >> 16, f.size)
        f.decode_span_device(vstart, vend, digest=False)


N_SIMD = 1024          # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
N_CU = 256
VALU_CYCLES = 2        # a wave64 VALU instruction holds its SIMD-32 2 cycles (MI355X_MICROARCH.md, wave scheduling)
SALU_PER_CU_CYCLE = 1  # one scalar ALU per CU


PMC_PASSES = (  # one rocprofv3 --pmc run each (FETCH_SIZE / WRITE_SIZE use 3 / 2 of the 4 TCC slots)
    ("fetch", ["FETCH_SIZE"]),
    ("write", ["WRITE_SIZE"]),
    ("issue", ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
               "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"]),
)


def pmc_traffic(path, vstart, vend, kernel):
    """Counters per launch of `kernel` (every full-size dispatch of it,
    whatever its template instance): one rocprofv3 --pmc pass per group of
    PMC_PASSES over a child process decoding the same split once.
    HBM bytes: corrections per MI355X_MICROARCH.md 'HBM [CDNA4]' (both
    counters are KiB; FETCH_SIZE counts half of a wide streaming read on
    gfx950, so it is doubled).  Issue: wave-instructions per launch against
    the cycles the launch held the chip (GRBM_GUI_ACTIVE is summed over the
    8 XCDs, so / 8): VALU capacity N_SIMD / VALU_CYCLES per cycle, SALU one
    per CU per cycle."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    sys.path.insert(0, os.path.join(ROOT, "profiles"))
    import summarize
    out, tot = {}, {}
    base = tempfile.mkdtemp(prefix="hbam_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    for sub, counters in PMC_PASSES:
        cmd = [prof, "--pmc"] + counters + ["--output-format", "csv", "-d", os.path.join(base, sub), "-o", "run",
                                            "--", sys.executable, os.path.abspath(__file__), "--pmc-child", path,
                                            "--pmc-span", str(vstart), str(vend)]
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                             start_new_session=True)
        try:
            _, err = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            p.wait()
            return {"error": f"{sub} pass timed out"}
        if p.returncode != 0:
            return {"error": f"{sub} pass rc={p.returncode}: {err.decode(errors='replace')[-300:]}"}
        cs = summarize.counters(base, sub, merge_instances=True)
        if sub in ("fetch", "write"):
            tot[sub] = summarize.totals(base, sub)
        e = cs.get(kernel)
        if not e:
            return {"error": f"{sub}: no dispatch of {kernel} in the counter file"}
        for c in counters:
            if "main:" + c in e:
                out[c] = e["main:" + c]
        out.setdefault("main_dispatches", e.get("main_dispatches"))
    shutil.rmtree(base, ignore_errors=True)
    if "FETCH_SIZE" not in out or "WRITE_SIZE" not in out:
        return {"error": "FETCH_SIZE / WRITE_SIZE missing from the counter files"}
    fetch = out["FETCH_SIZE"] * 1024 * 2
    write = out["WRITE_SIZE"] * 1024
    res = {"bytes_per_launch": int(fetch + write), "fetch_bytes": int(fetch), "write_bytes": int(write),
           "main_dispatches": out.get("main_dispatches")}
    # the child decodes the split once: every dispatch of its run summed is
    # one pass's HBM traffic (+ the open's few header-read dispatches)
    per = {}
    for k in set(tot.get("fetch", {})) | set(tot.get("write", {})):
        f_ = tot.get("fetch", {}).get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2
        w_ = tot.get("write", {}).get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        per[k] = (int(f_), int(w_))
    res["pass_traffic"] = {"bytes": sum(a + b for a, b in per.values()),
                           "per_kernel_GB": {k: round((a + b) / 1e9, 4) for k, (a, b) in
                                             sorted(per.items(), key=lambda kv: -sum(kv[1]))[:12]},
                           "kernel_bytes": {k: a + b for k, (a, b) in per.items()}}
    cyc = out.get("GRBM_GUI_ACTIVE", 0) / 8.0
    if cyc > 0 and "SQ_INSTS_VALU" in out:
        valu, salu = out["SQ_INSTS_VALU"], out.get("SQ_INSTS_SALU", 0.0)
        res["issue"] = {
            "valu_insts_per_launch": int(valu), "salu_insts_per_launch": int(salu),
            "lds_insts_per_launch": int(out.get("SQ_INSTS_LDS", 0)),
            "lds_bank_conflict_per_lds_inst": round(out.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                    max(out.get("SQ_INSTS_LDS", 0), 1), 3),
            "waves_per_launch": int(out.get("SQ_WAVES", 0)), "cycles_per_launch": int(cyc),
            "valu_frac": round(valu * VALU_CYCLES / (N_SIMD * cyc), 4),
            # LDS-array cycles (SQ_LDS_IDX_ACTIVE: every cycle the array serves a
            # wave-instruction, conflicts included) against one array per CU
            "lds_idx_active_per_launch": int(out.get("SQ_LDS_IDX_ACTIVE", 0)),
            "lds_cycles_per_lds_inst": round(out.get("SQ_LDS_IDX_ACTIVE", 0) / max(out.get("SQ_INSTS_LDS", 0), 1), 3),
            "lds_frac": round(out.get("SQ_LDS_IDX_ACTIVE", 0) / (N_CU * cyc), 4),
            "wait_inst_lds_frac_of_wave_cycles": round(out.get("SQ_WAIT_INST_LDS", 0) /
                                                       max(out.get("SQ_WAVE_CYCLES", 0), 1), 4),
            "salu_frac": round(salu / (N_CU * SALU_PER_CU_CYCLE * cyc), 4),
            "rule": f"valu_frac = SQ_INSTS_VALU x {VALU_CYCLES} cycles / ({N_SIMD} SIMDs x cycles); salu_frac = "
                    f"SQ_INSTS_SALU / ({N_CU} CUs x cycles); lds_frac = SQ_LDS_IDX_ACTIVE / ({N_CU} CUs x cycles); "
                    f"cycles = GRBM_GUI_ACTIVE / 8 (XCDs) of the launch"}
    return res


# ---------------------------------------------------------------------------
# side legs (N=1, rank 0)
# ---------------------------------------------------------------------------
def dropin_leg(path, first, records, short=False):
    """The call a JVM makes (hbam.h): hbam_open(path) maps the file (with
    opts.batch_records = the batch size, as GpuBAMRecordReader passes it, so
    the page-locked batch slots are pinned on a helper thread from the open
    on); each hbam_decode_span batch copies its windows host->HBM, decodes
    them and copies the 15 SoA columns plus the rest-of-record bytes into
    pinned host memory (BAMRecordReader.nextKeyValue's data).  Each batch
    size opens the split twice in this process: the first open allocates its
    page-locked batch buffers (device blocks may come from the process cache,
    hbam_mem.h, filled by the decodes before), the second finds both cached
    -- the case of an executor that reads many splits.  seconds = the batch
    loop; open_seconds = the hbam_open before it (header read).  short: the
    1 M-record batches only (the later placements of the leg)."""
    import hbam
    res = {}
    for label, batch in ((("batches_64K", 1 << 16),) if not short else ()) + (("batches_1M", 1 << 20),):
        for run in ("first_open", "second_open"):
            t0 = time.perf_counter()
            with hbam.BamFile(path=path, batch_records=batch) as f:
                t = time.perf_counter()
                n, k, nbytes = f.scan_batches(first, ALL, batch)
                dt = time.perf_counter() - t
                u = f.file_stats()[1]
            assert n == records, (n, records)
            res.setdefault(label, {})[run] = {
                "records": n, "batches": k, "rest_bytes_to_host": nbytes, "seconds": round(dt, 3),
                "open_seconds": round(t - t0, 4),
                "uncompressed_GBps": round(u / dt / 1e9, 3), "records_per_s": round(n / dt, 1)}
    if short:
        return res
    # the same 1 M-record loop with the file read through hbam_open_reader (a
    # positioned-read callback, as a Hadoop FSDataInputStream through JNI):
    # here os.pread in Python, one call at a time
    fd = os.open(path, os.O_RDONLY)
    try:
        size = os.fstat(fd).st_size
        for run in ("first_open", "second_open"):
            with hbam.BamFile(reader=lambda off, n: os.pread(fd, n, off), size=size, parallel_reads=True,
                              batch_records=1 << 20) as f:
                t = time.perf_counter()
                n, k, nbytes = f.scan_batches(first, ALL, 1 << 20)
                dt = time.perf_counter() - t
                u = f.file_stats()[1]
            assert n == records, (n, records)
            res.setdefault("batches_1M_reader_callback", {})[run] = {
                "records": n, "batches": k, "seconds": round(dt, 3), "uncompressed_GBps": round(u / dt / 1e9, 3),
                "records_per_s": round(n / dt, 1)}
        res["batches_1M_reader_callback"]["note"] = ("hbam_open_reader over os.pread (a Python callback, "
                                                     "parallel_reads: the copy threads call it at once) instead "
                                                     "of hbam_open's mapped path")
    finally:
        os.close(fd)
    return res


def pinned_host_leg(path, records):
    """SURVEY 8d's end-to-end from pinned host memory: the compressed file in
    page-locked host memory, copied host->HBM in 256 MiB pieces on a copy
    stream while the pieces already resident are located and inflated
    (hbam_gpu_run_streamed), then chain + decode + keys + voffs; records
    left in HBM."""
    import numpy as np
    import hbam
    data = np.fromfile(path, np.uint8)
    g = hbam.Gpu(0)
    try:
        with hbam.PinnedBuffer(data.nbytes) as buf:
            buf.array[:] = data
            g.load(data)
            del data
            piece = 256 << 20  # 64 MiB: 92 GB/s U, 256 MiB: 98 GB/s U on C2
            g.run_streamed(buf.ptr, buf.nbytes, piece)  # warm-up
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                st = g.run_streamed(buf.ptr, buf.nbytes, piece)
                ts.append(time.perf_counter() - t)
            assert st["records"] == records, (st["records"], records)
            u = st["inflated_bytes"]
    finally:
        g.close()
    dt = min(ts)
    return {"seconds": round(dt, 4), "uncompressed_GBps": round(u / dt / 1e9, 3),
            "records_per_s": round(records / dt, 1), "compressed_GBps_h2d": round(os.path.getsize(path) / dt / 1e9, 3)}


C3_SEG_RECORDS = 5_000_000  # records per segment of the C3 file
C3_BODIES = 3                # distinct body segments (each repeated an odd number of times)
# BASELINE config 3: "30x WGS-scale BAM (~600M reads, ~60 GB)".  The C2 model's
# unbinned qualities make ~141 B per record, which would put 600 M reads at
# ~85 GB; with Illumina's 8-level quality binning (gen_synth_bam.c mode 2)
# a record is ~100 B, so a ~60 GB file holds ~600 M reads: both figures.
C3_MODE = "wgs"


def c3_sequence(k):
    """Order of the body segments of the C3 file: k (about) copies spread
    over C3_BODIES distinct bodies, each an odd number of times, in a fixed
    shuffled order (no period: an error repeated in every copy of a body still
    moves the order-sensitive digests)."""
    import random
    counts = [k // C3_BODIES + (1 if j < k % C3_BODIES else 0) for j in range(C3_BODIES)]
    counts = [c if c % 2 else c + 1 for c in counts]
    seq = [j + 1 for j in range(C3_BODIES) for _ in range(counts[j])]
    random.Random(0x4842).shuffle(seq)
    return seq


def build_c3_file(path, D, target_gb, seg_records=C3_SEG_RECORDS):
    """The C3 BAM (~target_gb): a header segment then body segments (records
    [jS, (j+1)S) of a (1 + C3_BODIES) * S record model, S = C3_SEG_RECORDS)
    in c3_sequence order, then the EOF block.  Rank r generates the distinct
    segments j with j % world == r and writes every copy of them."""
    import numpy as np
    from hbam import synth
    t = time.time()
    n_model = (1 + C3_BODIES) * seg_records
    mine = {}
    for j in range(1 + C3_BODIES):
        if j % D.world == D.rank:
            mine[j] = synth.make_bam_segment(n_model, j * seg_records, (j + 1) * seg_records,
                                             with_header=j == 0, eof_block=False, seed=SEED + 3, mode=C3_MODE)
    sizes = {}
    for part in D.all_gather({j: (int(a.nbytes), int(i["uncompressed"])) for j, (a, i) in mine.items()}):
        sizes.update(part)
    body_mean = sum(sizes[j][0] for j in range(1, 1 + C3_BODIES)) / C3_BODIES
    k = max(1, int(-(-(target_gb * 1e9 - sizes[0][0]) // body_mean)))
    seq = c3_sequence(k)
    place = [(0, 0)]
    off = sizes[0][0]
    for j in seq:
        place.append((j, off))
        off += sizes[j][0]
    size = off + len(BGZF_EOF)
    if D.rank == 0:
        with open(path, "wb") as fh:
            fh.truncate(size)
    D.barrier()
    fd = os.open(path, os.O_WRONLY)
    try:
        for j, o in place:
            if j in mine:
                pwrite_all(fd, mine[j][0], o)
        if D.rank == 0:
            pwrite_all(fd, np.frombuffer(BGZF_EOF, np.uint8), off)
    finally:
        os.close(fd)
    del mine
    D.barrier()
    u = sizes[0][1] + sum(sizes[j][1] for j in seq)
    counts = {j: seq.count(j) for j in range(1, 1 + C3_BODIES)}
    meta = {"compressed_bytes": size, "uncompressed_bytes": u, "records": seg_records * (1 + len(seq)),
            "layout": f"header segment + {len(seq)} body segments of {seg_records} records: "
                      f"{C3_BODIES} distinct bodies x {counts} copies (odd), shuffled order, + EOF",
            "build_seconds": round(time.time() - t, 1)}
    log(f"[rank {D.rank}] C3 file {size} B, {meta['records']} records ({meta['build_seconds']}s)")
    return meta


def compose_digests(parts):
    """[(records, key_digest, voff_digest)] of consecutive spans -> the whole
    run's (records, key_digest, voff_digest) (hbam.h HBAM_DIGEST_P)."""
    n, kd, vd = 0, 0, 0
    for k, a, b in parts:
        w = pow(0x100000001B3, int(k), 1 << 64)
        kd = (kd * w + int(a)) & ALL
        vd = (vd * w + int(b)) & ALL
        n += int(k)
    return n, kd, vd


def bound_of(limits):
    """roofline.bound from the measured limits (fractions of each unit's
    peak): the largest one's unit when it reaches BOUND_MIN, else "latency"
    (no unit saturated: the kernel's dependent chain sets its pace)."""
    top = max(limits, key=limits.get)
    return top.replace("hbm_traffic", "hbm") if limits[top] >= BOUND_MIN else "latency"


def roofline_of(stats, world=1):
    """The roofline object of the dominant kernel from measurement passes
    (every inflate launch between its own HIP events on one stream: kernel
    durations, as rocprofv3 reports them)."""
    st = stats[-1]
    n_launch = max(1, st["inflate_launches"])
    avg = lambda k: sum(s_[k] for s_ in stats) / len(stats)
    kt = {"hbam::k_inflate_huff": avg("ms_huff"), "hbam::k_inflate_lz77": avg("ms_lz77"),
          "hbam::k_huff_tables": avg("ms_tables")}
    dom = max(kt, key=kt.get)
    dom_ms = kt[dom]
    if dom != "hbam::k_inflate_lz77":  # phase A launches once per round of each chunk
        n_launch *= INFLATE_ROUNDS
    b_alg = st["compressed_bytes"] + st["inflated_bytes"] + SOA_BYTES_PER_RECORD * st["records"]
    achieved = b_alg / (dom_ms * 1e-3) / 1e9
    # "unmeasured" until the in-session PMC passes (main()) set limits / bound:
    # the kernel's binding unit is a measured claim, never a default
    return {"bound": "unmeasured", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "launches_per_pass": n_launch, "avg_launch_ms": round(dom_ms / n_launch, 4),
            "alg_bytes_per_launch": int(b_alg / n_launch),
            "alg_bytes_rule": "(C + U + 37 N) of the pass / launches (SURVEY 8d)" +
                              ("" if world == 1 else ", rank 0's split"),
            "kernel_ms_per_pass": {k: round(v, 3) for k, v in kt.items()},
            "whole_pass": {"achieved": round(b_alg / (st["ms_total"] * 1e-3) / 1e9, 2),
                           "frac": round(b_alg / (st["ms_total"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}}


def run_c3(D, target_gb, steps, warmup, host_leg=False, solo=False):
    """C3 / C5 (strong scaling): the ranks split ONE ~60 GB BAM by BGZF byte
    ranges (hbam/shard.py: BAMInputFormat.addProbabilisticSplits on the GPU
    guesser), prefetch their split's bytes to HBM and time `steps` decodes of
    it; then, untimed: one measurement pass (stage / kernel times), a digest
    pass (order-sensitive key / voff digests composed in split order), and the
    .splitting-bai entries of each split at g = 4096 from the global record
    ordinals (hbam_splitting_entries), gathered on rank 0.  Rank 0 checks
    both against the oracle run over the whole file on every usable core.
    host_leg (N=1): first a decode with the windows copied from the mapped
    file inside the timed call (PCIe-inclusive)."""
    import numpy as np
    import hbam
    from hbam import shard
    path = os.path.join(scratch_dir(), f"hbam_c3_{D.tag}.bam")
    try:
        meta = build_c3_file(path, D, target_gb)
        size = meta["compressed_bytes"]
        res = {"file": meta}
        f = hbam.BamFile(path=path, device=D.device)
        first = f.header()["first_record_voff"]
        split = shard.ShardedBamReader(f, size, first, D.rank, D.world, D.all_gather).split()
        vs, ve = split if split is not None else (0, 0)
        lo, hi = vs >> 16, min(size, (ve >> 16) + (256 << 10))
        if host_leg:
            # feed-inclusive: every rank decodes its split with the windows
            # copied from the mapped file inside the timed call (the PCIe H2D
            # of its own bytes included), max over ranks
            D.barrier()
            t = time.perf_counter()
            st = f.decode_span_device(vs, ve, timing=False, digest=False) if split is not None else None
            dt_mine = time.perf_counter() - t
            D.barrier()
            dt = D.max_over_ranks(dt_mine)
            recs = D.all_gather(0 if st is None else int(st["records"]))
            res["c3_streamed_from_host"] = {
                "seconds": round(dt, 3), "uncompressed_GBps": round(meta["uncompressed_bytes"] / dt / 1e9, 3),
                "records_per_s": round(sum(recs) / dt, 1), "windows_rank0": None if st is None else st["windows"],
                "rank0_seconds": round(dt_mine, 3),
                "note": "each rank's split decoded with its windows copied from the mapped file (pageable, "
                        "through the host feed) inside the timed call; max over ranks"}
        t = time.perf_counter()
        if split is not None:
            f.prefetch(lo, hi)  # inputs resident in HBM before the timed region
        pf = time.perf_counter() - t
        log(f"[rank {D.rank}] C3 split [{vs:#x}, {ve:#x}) -> bytes [{lo}, {hi}) resident ({pf:.1f}s)")

        def step(timing=False, digest=False):
            return f.decode_span_device(vs, ve, timing=timing, digest=digest) if split is not None else None

        for _ in range(warmup):
            step()
        D.barrier()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        D.barrier()
        elapsed = D.max_over_ranks(time.perf_counter() - t)
        meas = step(timing=True)
        dig = step(digest=True)
        mine = (0, 0, 0) if dig is None else (int(dig["records"]), int(dig["key_digest"]), int(dig["voff_digest"]))
        parts = D.all_gather(mine)
        n_all, kd, vd = compose_digests(parts)
        base = sum(p[0] for p in parts[:D.rank])
        if split is not None:
            nrec, ent = f.splitting_entries(vs, ve, 4096, base)
            assert nrec == mine[0], (nrec, mine[0])
        else:
            ent = np.zeros(0, np.uint64)
        gathered = D.all_gather(ent.tobytes())
        f.close()
        solo_res = None
        if solo and D.world > 1:
            # the N = 1 figure of this same workload: rank 0 decodes the whole
            # file alone (resident, same steps), the other ranks wait
            if D.rank == 0:
                g = hbam.BamFile(path=path, device=D.device)
                try:
                    whole = (first, (size << 16) | 0xFFFF)
                    t = time.perf_counter()
                    g.prefetch(first >> 16, size)
                    pf1 = time.perf_counter() - t
                    g.decode_span_device(*whole, digest=False)
                    ns = max(1, min(steps, 5))
                    t = time.perf_counter()
                    for _ in range(ns):
                        st1 = g.decode_span_device(*whole, digest=False)
                    dt1 = time.perf_counter() - t
                finally:
                    g.close()
                solo_res = {"value": meta["uncompressed_bytes"] * ns / dt1 / 1e9, "ms_per_step": dt1 / ns * 1e3,
                            "steps": ns, "records": int(st1["records"]), "prefetch_seconds": round(pf1, 2),
                            "note": "rank 0 alone decoding the whole C3 file (resident in its HBM) while the "
                                    "other ranks wait: the N = 1 value of this workload"}
            D.barrier()
        if D.rank != 0:
            return None
        sbi = shard.be64([first]) + b"".join(
            np.frombuffer(g, np.uint64).astype(">u8").tobytes() for g in gathered) + shard.be64([size << 16])
        u = meta["uncompressed_bytes"]
        res.update({
            "value": u * steps / elapsed / 1e9, "ms_per_step": elapsed / steps * 1e3,
            "records_per_s": meta["records"] * steps / elapsed, "records": n_all,
            "split_bytes_rank0": hi - lo, "prefetch_seconds_rank0": round(pf, 3),
            "stages_ms_rank0": None if meas is None else {
                k: round(meas[k], 3) for k in ("ms_locate", "ms_inflate", "ms_tables", "ms_huff", "ms_lz77",
                                               "ms_chain", "ms_decode", "ms_total")},
            "windows_rank0": None if meas is None else meas["windows"],
            "roofline": None if meas is None else roofline_of([meas], D.world)})
        # the oracle over the whole file (rank 0, every usable core)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import orc
        cores = host_cores()
        data = np.memmap(path, np.uint8, mode="r", shape=(size,))
        t = time.perf_counter()
        dec, _ = orc.scan(data, threads=cores, mode="decode")
        dto = time.perf_counter() - t
        t = time.perf_counter()
        ires, want = orc.scan(data, threads=cores, mode="index", granularity=4096)
        dtoi = time.perf_counter() - t
        del data
        res["c3_parity"] = {
            "records": n_all == dec["records"] == meta["records"],
            "key_digest": kd == dec["key_digest"], "voff_digest": vd == dec["voff_digest"],
            "digest": "order-sensitive (HBAM_DIGEST_P), composed over the ranks' splits in file order",
            "oracle_seconds": round(dto, 1), "oracle_threads": cores,
            "oracle_uncompressed_GBps": round(u / dto / 1e9, 3)}
        res["c5_splitting_bai_g4096"] = {
            "entries": len(sbi) // 8, "identical_to_oracle": sbi == want,
            "assembled_from": f"{D.world} split(s): hbam_splitting_entries per rank, gathered on rank 0",
            "oracle_seconds": round(dtoi, 1), "oracle_threads": cores}
        res["matches_oracle"] = bool(res["c3_parity"]["records"] and res["c3_parity"]["key_digest"] and
                                     res["c3_parity"]["voff_digest"] and
                                     res["c5_splitting_bai_g4096"]["identical_to_oracle"])
        model = cpu_model()
        res["cpu_baseline"] = {
            "value": round(u / dto / 1e9, 4), "unit": "GB/s", "cores": cores, "kind": "port",
            "host_cores_total": os.cpu_count(), "records_per_s": round(dec["records"] / dto, 1), "cpu_model": model,
            "sample": f"whole C3 file ({u} inflated bytes, {dec['records']} records) through oracle/orc_scan.c "
                      f"(system zlib, htsjdk reader rules, STRICT) on {cores} threads of rank 0's host "
                      f"({model}), {dto:.1f} s"}
        res["solo"] = solo_res
        return res
    finally:
        D.barrier()
        if D.rank == 0:
            try:
                os.unlink(path)
            except OSError:
                pass


def long_read_leg():
    """C4-like: ONT-style 10-50 kb reads (records spanning many blocks, heavy
    aux tags), resident, through the same device pipeline."""
    import hbam
    from hbam import synth
    data, info = synth.make_bam(12000, mode="long", as_numpy=True, seed=SEED + 4)
    g = hbam.Gpu(0)
    try:
        g.load(data)
        g.run()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            g.run()
            ts.append(time.perf_counter() - t)
        st = g.run(timing=True)  # untimed measurement pass: per-stage times
    finally:
        g.close()
    dt = min(ts)
    return {"records": int(st["records"]), "compressed_bytes": info["compressed"],
            "uncompressed_bytes": info["uncompressed"], "seconds": round(dt, 5),
            "uncompressed_GBps": round(info["uncompressed"] / dt / 1e9, 3),
            "stages_ms": {k: round(st[k], 3) for k in ("ms_locate", "ms_huff", "ms_lz77", "ms_chain", "ms_decode")}}


def write_legs(path, size, info_u):
    """SAMRecordWritable.write of the decoded file on the GPU, the measured
    D2D copy ceiling, and the BGZF write path (the inflated file recompressed
    at level 5 with its own block boundaries, byte-identical to the file)."""
    import zlib
    import numpy as np
    import hbam
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    data = np.fromfile(path, np.uint8)
    g = hbam.Gpu(0)
    res = {}
    try:
        g.load(data)
        g.run()
        ms, nb = g.encode_writables(iters=10)
        d2d = g.d2d_bandwidth(1 << 32, 5)
        res["writable_encode"] = {
            "bytes": nb, "ms": round(ms, 4), "GBps_encoded": round(nb / ms / 1e6, 2),
            "roofline": {"bound": "unmeasured", "achieved": round(2 * nb / ms / 1e6, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(2 * nb / ms / 1e6 / HBM_PEAK_GBS, 4)},
            "frac_of_measured_d2d": round(2 * nb / ms / 1e6 / d2d, 4)}
        res["d2d_copy_GBps_measured"] = round(d2d, 1)
        g.bgzf_compress(level=5, eof=False, iters=0)
        ms, nbw = g.bgzf_compress(level=5, eof=False, iters=1)
        same = nbw == data.nbytes and bool(np.array_equal(g.fetch_compressed(0, nbw), data))
    finally:
        g.close()
    cores = host_cores()
    nblk = 200 * cores  # 200 blocks per thread in the all-cores sample
    raw = data[:min(data.nbytes, nblk * 65536 * 2)].tobytes()
    p, pay, lens = 0, [], []
    while len(lens) < nblk and p + 18 <= len(raw):
        bs = int.from_bytes(raw[p + 16:p + 18], "little") + 1
        if p + bs > len(raw):
            break
        x = zlib.decompressobj(-15).decompress(raw[p + 18:p + bs - 8])
        pay.append(x)
        lens.append(len(x))
        p += bs
    one = b"".join(pay[:200])
    t = time.perf_counter()
    orc.bgzf_compress(one, lens[:200], level=5, eof=False)
    dt = time.perf_counter() - t
    # every usable core: thread j compresses blocks [200 j, 200 j + 200) of the
    # sample (orc_bgzf_compress releases the GIL inside ctypes)
    from concurrent.futures import ThreadPoolExecutor
    parts = [(b"".join(pay[j:j + 200]), lens[j:j + 200]) for j in range(0, len(lens), 200)]
    t = time.perf_counter()
    with ThreadPoolExecutor(max_workers=cores) as ex:
        list(ex.map(lambda a: orc.bgzf_compress(a[0], a[1], level=5, eof=False), parts))
    dt_all = time.perf_counter() - t
    n_all = sum(len(a[0]) for a in parts)
    res["bgzf_write"] = {
        "level": 5, "ms": round(ms, 2), "uncompressed_GBps": round(info_u / ms / 1e6, 4),
        "identical_to_file": same, "bytes_out": int(nbw),
        "cpu_baseline": {"value": round(n_all / dt_all / 1e9, 5), "unit": "GB/s", "cores": cores, "kind": "port",
                         "sample": f"first {len(lens)} blocks ({n_all} B) through oracle orc_bgzf_compress "
                                   f"(system zlib, level 5), {len(parts)} ranges of 200 blocks on {cores} threads, "
                                   f"{dt_all:.2f} s",
                         "single_thread": {"value": round(len(one) / dt / 1e9, 5), "unit": "GB/s", "cores": 1,
                                           "sample": f"first 200 blocks ({len(one)} B), {dt:.2f} s"}}}
    return res


# ---------------------------------------------------------------------------
class Dist:
    """One process per GPU (torchrun env); torch.distributed (RCCL on GPUs)
    only for metadata all_gathers, barriers and the timing all_reduce."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.device = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = args.dist_backend
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            if not args.dry_run:
                torch.cuda.set_device(self.device)
            dist.init_process_group(self.backend)
            self.dist = dist
        self.tag = self.all_gather(f"{os.getpid()}_{int(time.time())}")[0]

    def all_gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def barrier(self):
        # hbam calls return after their streams drain; torch's stream is idle
        if self.dist is not None:
            import torch
            torch.cuda.synchronize()
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64,
                         device=f"cuda:{self.device}" if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def run_c2(D, args, steps, warmup, extras):
    """C2 (N=1) / N x C2 weak scaling: every rank decodes one C2 of records
    from its split of one shared file.  extras (N=1): the CPU baseline, PMC
    traffic and the side legs, on the same file."""
    import hbam
    from hbam import shard
    path = os.path.join(scratch_dir(), f"hbam_bench_{D.tag}.bam")
    try:
        size, u_file = build_shared_bam(path, D.rank, D.world, args.records, D.all_gather, D.barrier)
        f = hbam.BamFile(path=path, device=D.device)
        first = f.header()["first_record_voff"]
        split = shard.ShardedBamReader(f, size, first, D.rank, D.world, D.all_gather).split()
        vs, ve = split if split is not None else (0, 0)
        lo = vs >> 16
        hi = min(size, (ve >> 16) + (256 << 10))
        if split is not None:
            f.prefetch(lo, hi)  # inputs resident in HBM before the timed region
        log(f"[rank {D.rank}] split [{vs:#x}, {ve:#x}) -> bytes [{lo}, {hi}) resident")

        def step(timing=True, digest=False):
            if split is None:
                return None
            return f.decode_span_device(vs, ve, timing=timing, digest=digest)

        for _ in range(warmup):
            step(timing=args.serial)
        D.barrier()
        t = time.perf_counter()
        for _ in range(steps):
            step(timing=args.serial)  # production launch order (phase A / phase B overlapped), no events
        D.barrier()
        elapsed = D.max_over_ranks(time.perf_counter() - t)
        # untimed measurement passes: every launch on one stream between its own
        # HIP events -> per-stage and per-kernel durations (the roofline)
        stats = [step(timing=True) for _ in range(3)]
        tokens = f.inflate_token_count() if split is not None else 0  # phase A's output of that pass
        check = step(timing=args.serial, digest=True)  # untimed: the digests for the parity check
        mine = (0, 0, 0, 0) if check is None else (int(check["records"]), int(check["inflated_bytes"]),
                                                   int(check["key_digest"]), int(check["voff_digest"]))
        parts = D.all_gather(mine)
        n_all, kd, vd = compose_digests([(p[0], p[2], p[3]) for p in parts])
        u_all = sum(p[1] for p in parts)
        assert n_all == D.world * args.records, (n_all, D.world * args.records)
        solo = None
        if D.world > 1 and not args.no_solo:
            # the N = 1 figure: rank 0 decodes its own split (one C2) alone
            if D.rank == 0 and split is not None:
                step(timing=args.serial)
                t = time.perf_counter()
                for _ in range(steps):
                    step(timing=args.serial)
                dt = time.perf_counter() - t
                solo = {"value": round(mine[1] * steps / dt / 1e9, 3), "ms_per_step": round(dt / steps * 1e3, 3),
                        "note": "rank 0 alone decoding its split (one C2) while the other ranks wait"}
            D.barrier()
        out = None
        if D.rank == 0:
            st = stats[-1] if stats and stats[-1] is not None else check
            value = u_all * steps / elapsed / 1e9
            out = {
                "value": value, "ms_per_step": elapsed / steps * 1e3,
                "per_gpu_value": round(value / D.world, 3),
                "scaling_detail": None if solo is None else {
                    "solo_value": solo["value"], "solo": solo,
                    "efficiency_vs_solo": round(value / (D.world * solo["value"]), 4),
                    "rule": "value / (N x solo_value): N splits of one C2 each decoded concurrently against "
                            "rank 0's split decoded alone"},
                "records_per_s": n_all * steps / elapsed,
                "config": {"workload": ("C2: synthetic 10M x 150bp paired-end coordinate-sorted BAM" if D.world == 1
                                        else f"N x C2: one BAM of {D.world} x C2 records split by BGZF ranges "
                                             f"(weak scaling)"),
                           "records_per_gpu": args.records, "file_bytes": size, "uncompressed_bytes": u_file,
                           "split_bytes_rank0": hi - lo,
                           "parallelism": f"FileVirtualSplit per rank x{D.world} (BAMSplitGuesser)"},
                "parity": {"records": n_all, "key_digest": f"{kd:#018x}", "voff_digest": f"{vd:#018x}"},
                "link_fallbacks": int(sum(s_["link_fallbacks"] for s_ in stats)),
                "link_rewalks": int(sum(s_["link_rewalks"] for s_ in stats)),
                "stages_ms": {k: round(st[k], 3) for k in ("ms_locate", "ms_inflate", "ms_tables", "ms_huff",
                                                            "ms_lz77", "ms_chain", "ms_decode", "ms_total")},
                "roofline": roofline_of(stats, D.world),
                "cpu_baseline": None,
            }
        f.close()
        if D.rank == 0 and extras:
            if not args.no_cpu_baseline:
                try:
                    cb, full = cpu_baseline(path, size, args.cpu_seconds)
                    out["cpu_baseline"] = cb
                    out["parity"]["matches_oracle"] = bool(full["records"] == n_all and full["key_digest"] == kd
                                                           and full["voff_digest"] == vd)
                except Exception as e:  # reported, never substituted for the GPU number
                    out["cpu_baseline"] = {"error": repr(e)}
            extra = {}
            want = (lambda name: not args.no_extra and (args.extras is None or name in args.extras.split(",")))
            if want("dropin_end_to_end"):
                # before the PMC child runs: after them (as after hbam_gpu_run_streamed,
                # main()), the drop-in loop of this process ran at 24 instead of
                # 39-40 GB/s U on first open (open issue)
                t = time.time()
                try:
                    extra["dropin_end_to_end"] = dropin_leg(path, first, n_all)
                except Exception as e:
                    extra["dropin_end_to_end"] = {"error": repr(e)}
                log(f"[extra] dropin_end_to_end {time.time() - t:.1f}s")
            if not args.no_pmc:
                try:
                    st_c = stats[-1]["compressed_bytes"]
                    tr = pmc_traffic(path, vs, ve, out["roofline"]["kernel"])
                    if tr and "bytes_per_launch" in tr:
                        rf = out["roofline"]
                        rf["traffic"] = tr["bytes_per_launch"]
                        rf["traffic_detail"] = {k: v for k, v in tr.items() if k not in ("issue", "pass_traffic")}
                        rf["traffic_detail"]["source"] = "rocprofv3 --pmc child runs, this session, every " \
                                                         "full-size dispatch of the kernel"
                        rf["traffic_frac_of_alg"] = round(tr["bytes_per_launch"] / max(rf["alg_bytes_per_launch"], 1), 3)
                        if "issue" in tr:
                            rf["issue"] = tr["issue"]
                            lim = {"hbm": rf["frac"], "valu_issue": tr["issue"]["valu_frac"],
                                   "salu_issue": tr["issue"]["salu_frac"], "lds": tr["issue"]["lds_frac"],
                                   "hbm_traffic": tr["bytes_per_launch"] / (rf["avg_launch_ms"] * 1e-3) / 1e9
                                   / HBM_PEAK_GBS}
                            rf["limits"] = {k: round(v, 4) for k, v in lim.items()}
                            rf["bound"] = bound_of(lim)
                            rf["bound_rule"] = (f"the largest of: algorithmic HBM bytes / peak (frac), measured "
                                                f"HBM traffic / peak, VALU and SALU issue fractions and the "
                                                f"LDS-array busy fraction (issue), when it is >= {BOUND_MIN}; "
                                                f"'latency' when every limit is below {BOUND_MIN} (no unit "
                                                f"saturated: the dependent chain sets the pace); "
                                                "achieved / peak / frac stay the algorithmic-bytes HBM figures")
                        pt = tr.get("pass_traffic")
                        if pt:
                            b_alg = rf["alg_bytes_per_launch"] * rf["launches_per_pass"]
                            wp = rf["whole_pass"]
                            wp["traffic"] = pt["bytes"]
                            wp["traffic_frac_of_alg"] = round(pt["bytes"] / max(b_alg, 1), 3)
                            wp["traffic_GBps"] = round(pt["bytes"] / (out["ms_per_step"] * 1e-3) / 1e9, 1)
                            wp["traffic_per_kernel_GB"] = pt["per_kernel_GB"]
                            wp["traffic_rule"] = ("FETCH_SIZE x 2 + WRITE_SIZE (KiB -> B) summed over every "
                                                  "dispatch of a child that decodes the split once, against "
                                                  "C + U + 37 N; traffic_GBps over the timed step")
                            ka = pt["kernel_bytes"].get("hbam::k_inflate_huff")
                            if ka and tokens:
                                a_alg = st_c + 4 * tokens
                                rf["phase_a"] = {
                                    "traffic": ka, "alg_bytes": a_alg, "traffic_frac_of_alg": round(ka / a_alg, 3),
                                    "tokens": tokens,
                                    "rule": "k_inflate_huff traffic of one pass (every dispatch) against its own "
                                            "algorithmic bytes: C read + 4 B per LZ77 token written"}
                    elif tr:
                        out["roofline"]["traffic_error"] = tr["error"]
                except Exception as e:
                    out["roofline"]["traffic_error"] = repr(e)
                if want("dropin_end_to_end"):
                    # the same loop again after the PMC child processes (DESIGN.md 7 item 5:
                    # some earlier GPU work slows a later drop-in loop of the process)
                    try:
                        extra["dropin_after_pmc"] = dropin_leg(path, first, n_all, short=True)
                    except Exception as e:
                        extra["dropin_after_pmc"] = {"error": repr(e)}
            if not args.no_extra:
                # (the pinned-host leg runs last of all, in main())
                for name, fn in (("write_path", lambda: write_legs(path, size, u_file)),
                                 ("c4_long_reads", long_read_leg)):
                    if not want(name):
                        continue
                    t = time.time()
                    try:
                        extra[name] = fn()
                    except Exception as e:
                        extra[name] = {"error": repr(e)}
                    log(f"[extra] {name} {time.time() - t:.1f}s")
                out["extra"] = extra
                d2d = (extra.get("write_path") or {}).get("d2d_copy_GBps_measured")
                if d2d:  # the read path against the measured device-to-device copy rate
                    rf = out["roofline"]
                    rf["measured_d2d_GBps"] = d2d
                    rf["frac_of_measured_d2d"] = round(rf["achieved"] / d2d, 5)
                    rf["whole_pass"]["frac_of_measured_d2d"] = round(rf["whole_pass"]["achieved"] / d2d, 5)
        return out
    finally:
        D.barrier()
        if D.rank == 0:
            try:
                os.unlink(path)
            except OSError:
                pass


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` with no launcher (WORLD_SIZE unset): start N rank
    processes of this script, one per GPU, with the env torchrun would give
    them (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), and wait for them.  The
    parent runs before anything imports torch or libhbam, so it never touches
    a GPU (no exec: the ranks are children).  The ranks inherit stdout, so rank
    0's JSON line is the one line printed.  If a rank fails, the others are
    stopped (their own PIDs) and the parent exits with the first failing code;
    a SIGTERM to the parent is passed on to the ranks."""
    import signal
    port = free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", ROLE_RANK="0", HBAM_BENCH_SPAWNED="1")
    procs = []

    def stop(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_term(signum, frame):
        stop()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    import threading

    def relay(pipe):
        # rank stdout: JSON lines (rank 0's result) to stdout, anything else
        # (gloo / RCCL chatter) to stderr, so stdout holds the one result line
        for line in iter(pipe.readline, b""):
            out = sys.stdout if line.lstrip().startswith(b"{") else sys.stderr
            out.buffer.write(line)
            out.flush()
        pipe.close()

    relays = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE))
        relays.append(threading.Thread(target=relay, args=(procs[-1].stdout,), daemon=True))
        relays[-1].start()
    rc = 0
    t_fail = None
    while True:
        alive = [p.poll() is None for p in procs]  # poll every rank (no short-circuit)
        if not any(alive):
            break
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad and t_fail is None:
            rc = bad[0]
            log(f"[bench] a rank exited with {rc}: stopping the others")
            stop()
            t_fail = time.time()
        elif t_fail is not None and time.time() - t_fail > 30:
            stop(signal.SIGKILL)
        time.sleep(0.2)
    for t in relays:
        t.join(timeout=10)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    return rc if rc >= 0 else 128 - rc


def check_world(args):
    """torchrun (or spawn_ranks) sets WORLD_SIZE: it must equal --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != args.gpus:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={ws}: pass --gpus equal to the number of ranks")
        sys.exit(2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c2", "c3"), default=None,
                    help="c2: C2 per rank (weak); c3: one ~60 GB BAM split over the ranks (strong). "
                         "Default: c2 at one GPU, c3 at N > 1")
    ap.add_argument("--records", type=int, default=10_000_000, help="C2 records per rank (10M)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-session rocprofv3 PMC passes")
    ap.add_argument("--no-extra", action="store_true", help="skip every side leg (drop-in, C3/C5, C4, write)")
    ap.add_argument("--extras", default=None,
                    help="comma list of the C2 side legs to run (dropin_end_to_end, write_path, "
                         "c4_long_reads, c2_from_pinned_host); default all")
    ap.add_argument("--serial", action="store_true",
                    help="every step in the measurement launch order (one stream, events per launch): the "
                         "command profiles/collect.sh traces, so rocprofv3's per-kernel averages are the "
                         "durations the roofline uses")
    ap.add_argument("--c3-gb", type=float, default=60.0, help="size of the C3/C5 file (0: skip the C3 side leg)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo + --one-device: rehearse the N-rank sequence on a one-GPU box")
    ap.add_argument("--one-device", action="store_true", help="every rank on device 0 (rehearsal only)")
    ap.add_argument("--no-solo", action="store_true",
                    help="N > 1: skip rank 0's solo pass (the N = 1 value of the same workload)")
    ap.add_argument("--no-feed-leg", action="store_true",
                    help="N > 1: skip the feed-inclusive C3 decode (windows copied from the mapped file)")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks and rendezvous (gloo), report them, decode nothing (CPU test of the launch)")
    ap.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-span", type=int, nargs=2, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.pmc_child:
        pmc_child(args.pmc_child, *args.pmc_span)
        return
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    check_world(args)
    if args.dry_run and os.environ.get("HBAM_BENCH_FAIL_RANK") == os.environ.get("RANK"):
        sys.exit(3)  # test hook: a rank that dies before the rendezvous

    D = Dist(args)
    if args.dry_run:  # the launch path alone (CPU tests): every rank reports, rank 0 prints
        ranks = D.all_gather({"rank": D.rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                              "world": D.world, "pid": os.getpid()})
        if D.rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": D.world, "ranks": ranks}), flush=True)
        D.close()
        return
    workload = args.workload or ("c2" if D.world == 1 else "c3")
    line = None
    if workload == "c2":
        r = run_c2(D, args, args.steps, args.warmup, extras=D.world == 1)
        if D.rank == 0:
            line = dict(r, scaling="weak", workload_key="c2")
        if D.world == 1 and not args.no_extra and args.c3_gb > 0:
            t = time.time()
            try:
                c3 = run_c3(D, args.c3_gb, steps=3, warmup=1, host_leg=True)
            except Exception as e:
                c3 = {"error": repr(e)}
            log(f"[extra] c3_c5_60GB {time.time() - t:.1f}s")
            if D.rank == 0:
                line.setdefault("extra", {})["c3_c5_60GB"] = c3
        if D.world == 1 and not args.no_extra and (args.extras is None or "c2_from_pinned_host" in args.extras):
            # last of all: after hbam_gpu_run_streamed has run in a process, the
            # drop-in loop of a later context ran at ~24 instead of ~40 GB/s U
            # (scripts/dropin_probe2.py --steps)
            t = time.time()
            path = os.path.join(scratch_dir(), f"hbam_pinned_{D.tag}.bam")
            try:
                size, _ = build_shared_bam(path, 0, 1, args.records, D.all_gather, D.barrier)
                ph = pinned_host_leg(path, args.records)
                if args.extras is None or "dropin_end_to_end" in args.extras:
                    # the drop-in loop once more, after hbam_gpu_run_streamed ran in this process
                    import hbam
                    with hbam.BamFile(path=path) as f:
                        first = f.header()["first_record_voff"]
                    line.setdefault("extra", {})["dropin_after_run_streamed"] = dropin_leg(path, first, args.records,
                                                                                         short=True)
            except Exception as e:
                ph = {"error": repr(e)}
            finally:
                if os.path.exists(path):
                    os.unlink(path)
            log(f"[extra] c2_from_pinned_host {time.time() - t:.1f}s")
            line.setdefault("extra", {})["c2_from_pinned_host"] = ph
    else:
        r = run_c3(D, args.c3_gb, args.steps, args.warmup, host_leg=not args.no_feed_leg, solo=not args.no_solo)
        if D.rank == 0:
            solo = r.get("solo")
            line = {"value": r["value"], "ms_per_step": r["ms_per_step"], "records_per_s": r["records_per_s"],
                    "per_gpu_value": round(r["value"] / D.world, 3),
                    "scaling_detail": None if not solo else {
                        "solo_value": round(solo["value"], 3), "solo": solo,
                        "efficiency_vs_solo": round(r["value"] / (D.world * solo["value"]), 4),
                        "rule": "value / (N x solo_value): the same C3 file, its N splits decoded concurrently "
                                "against rank 0 decoding all of it alone"},
                    "scaling": "strong", "workload_key": "c3",
                    "config": {"workload": f"C3: one {r['file']['compressed_bytes'] / 1e9:.1f} GB synthetic BAM "
                                           f"(150 bp paired-end model) split by BGZF byte ranges across "
                                           f"{D.world} GPU(s)",
                               "file_bytes": r["file"]["compressed_bytes"],
                               "uncompressed_bytes": r["file"]["uncompressed_bytes"],
                               "records": r["file"]["records"], "layout": r["file"]["layout"],
                               "split_bytes_rank0": r["split_bytes_rank0"],
                               "parallelism": f"FileVirtualSplit per rank x{D.world} (BAMSplitGuesser)"},
                    "parity": {"records": r["records"], "matches_oracle": r["matches_oracle"],
                               "c3": r["c3_parity"], "c5_splitting_bai_g4096": r["c5_splitting_bai_g4096"]},
                    "feed_inclusive": r.get("c3_streamed_from_host"),
                    "stages_ms": r["stages_ms_rank0"], "windows_rank0": r["windows_rank0"],
                    "roofline": r["roofline"], "cpu_baseline": r["cpu_baseline"]}
        if D.world > 1 and not args.no_extra:
            # the C3 contexts are closed: their cached device blocks go back to
            # HIP first (with --one-device the ranks share one GPU's HBM)
            import gc
            import hbam
            gc.collect()
            hbam.release_cached_memory()
            try:  # the weak-scaling side leg: N x C2, one C2 per rank
                w = run_c2(D, args, steps=max(3, args.steps // 2), warmup=1, extras=False)
            except Exception as e:
                log(f"[rank {D.rank}] weak N x C2 leg failed: {e!r}")
                w = {"error": repr(e)}
            if D.rank == 0:
                line["extra"] = {"weak_nxc2": w}
    if D.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(line.pop("value"), 3),
            "unit": "GB/s",
            "n_gpus": D.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(line.pop("ms_per_step"), 3),
            "higher_is_better": True,
            "scaling": line.pop("scaling"),
            "vs_baseline": None,
            "dtype": "u8",
            "launch_order": "serial (measurement)" if args.serial else "overlapped (production)",
            "env": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")},
            "data": "synthetic (tools/gen_synth_bam.c: Illumina-like qualities, zlib level 5 BGZF), "
                    "generated on the box",
        }
        line.pop("workload_key")
        line["records_per_s"] = round(line["records_per_s"], 1)
        out.update(line)
        print(json.dumps(out), flush=True)
    D.close()


if __name__ == "__main__":
    main()
