"""Rows of BASELINE.md section 3 from one bench.py JSON line (developer
script): python scripts/baseline_table.py profiles/r03_x/bench_default.json"""
import json
import sys

HBM = 8000.0


def row(cfg, path, who, c, u, n, t, frac=None):
    gbs = u / t / 1e9 if t else 0.0
    rps = n / t if t else 0.0
    f = f"{frac:.4f}" if frac is not None else "—"
    return f"| {cfg} | {path} | {who} | {c / 1e9:.3f} | {u / 1e9:.3f} | {n:,} | {t:.4f} | {gbs:.2f} | {rps / 1e6:.1f} M | {f} |"


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    cfg = d["config"]
    c2c, c2u = cfg["file_bytes"], cfg["uncompressed_bytes"]
    n = d["parity"]["records"]
    t = d["ms_per_step"] / 1e3
    b_alg = c2c + c2u + 37 * n
    rows = [row("C2", "MI355X, resident in HBM (timed steps)", "1 GPU", c2c, c2u, n, t, b_alg / t / 1e9 / HBM)]
    cb = d.get("cpu_baseline") or {}
    if "value" in cb:
        rows.append(row("C2", f"CPU oracle (orc_scan.c, zlib, STRICT), {cb.get('cpu_model', '')}",
                        f"{cb['cores']} threads (of {cb.get('host_cores_total', '?')})", c2c, c2u, n,
                        c2u / (cb["value"] * 1e9)))
        st = cb.get("single_thread") or {}
        if "value" in st:
            rows.append(f"| C2 | CPU oracle, one thread, prefix sample | 1 thread | — | — | — | — | {st['value']:.3f} | "
                        f"{st['records_per_s'] / 1e6:.2f} M | — |")
    ex = d.get("extra") or {}
    ph = ex.get("c2_from_pinned_host") or {}
    if "seconds" in ph:
        rows.append(row("C2", "MI355X, end to end from page-locked host memory", "1 GPU", c2c, c2u, n, ph["seconds"]))
    di = (ex.get("dropin_end_to_end") or {}).get("batches_1M") or {}
    for k in ("first_open", "second_open"):
        if k in di:
            rows.append(row("C2", f"MI355X, drop-in hbam_open(path) + hbam_decode_span 1M batches -> pinned host "
                                  f"({k.replace('_', ' ')})", "1 GPU", c2c, c2u, n, di[k]["seconds"]))
    for leg, where in (("dropin_after_pmc", "after the PMC child runs"),
                       ("dropin_after_run_streamed", "after hbam_gpu_run_streamed")):
        dj = (ex.get(leg) or {}).get("batches_1M") or {}
        for k in ("first_open", "second_open"):
            if k in dj:
                rows.append(row("C2", f"MI355X, drop-in 1M batches, {where} ({k.replace('_', ' ')})", "1 GPU",
                                c2c, c2u, n, dj[k]["seconds"]))
    c4 = ex.get("c4_long_reads") or {}
    if "seconds" in c4:
        rows.append(row("C4", "MI355X, resident", "1 GPU", c4["compressed_bytes"], c4["uncompressed_bytes"],
                        c4["records"], c4["seconds"]))
    c3 = ex.get("c3_c5_60GB") or {}
    if "file" in c3:
        f = c3["file"]
        rows.append(row("C3", "MI355X, resident (split of the whole file)", "1 GPU", f["compressed_bytes"],
                        f["uncompressed_bytes"], f["records"], c3["ms_per_step"] / 1e3))
        h = c3.get("c3_streamed_from_host") or {}
        if "seconds" in h:
            rows.append(row("C3", "MI355X, windows copied from the mapped file inside the timed call", "1 GPU",
                            f["compressed_bytes"], f["uncompressed_bytes"], f["records"], h["seconds"]))
        p = c3.get("c3_parity") or {}
        if "oracle_seconds" in p:
            rows.append(row("C3", "CPU oracle (orc_scan.c)", f"{p['oracle_threads']} threads", f["compressed_bytes"],
                            f["uncompressed_bytes"], f["records"], p["oracle_seconds"]))
    print("\n".join(rows))


if __name__ == "__main__":
    main()
