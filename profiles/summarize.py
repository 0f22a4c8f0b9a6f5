#!/usr/bin/env python3
"""Summarise one rocprofv3 collection (profiles/collect.sh) into JSON.

Input dir layout: <dir>/trace/**/run_kernel_stats.csv (kernel trace --stats),
<dir>/{fetch,write,sq}/**/run_counter_collection.csv (one PMC pass each).

Per kernel: calls, average duration (ns) and, from the PMC passes, average
FETCH_SIZE / WRITE_SIZE per dispatch converted to bytes.  "main_*" fields
average only the full-size dispatches of a kernel (grid >= half its largest
grid): the pipeline also launches tiny instances (header read), which would
otherwise skew a per-launch figure.  Corrections follow
/opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE/WRITE_SIZE are
kilobytes (counter_defs.yaml), and on gfx950 FETCH_SIZE reports half the bytes
of a wide coalesced streaming read, so it is doubled ("fetch_bytes_corrected").
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _find(d, name):
    hits = glob.glob(os.path.join(d, "**", name), recursive=True)
    return hits[0] if hits else None


def _col(row, *cands):
    for c in cands:
        if c in row:
            return row[c]
    for k in row:
        for c in cands:
            if k.lower() == c.lower():
                return row[k]
    raise KeyError(cands)


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    if "rocprim" in n:
        return "rocprim:" + ("scan" if "scan" in name else "sort" if "sort" in name else "other")
    # k_inflate_huff<STAGE, KEEP>: the default build (KEEP false) keeps the
    # round-1/2 names k_inflate_huff<true> / <false>
    return n.replace("void ", "").replace(", false>", ">").strip()


def kernel_stats(d):
    p = _find(os.path.join(d, "trace"), "*kernel_stats.csv")
    out = {}
    if not p:
        return out
    for r in csv.DictReader(open(p)):
        name = short(_col(r, "Name", "KernelName"))
        calls = int(_col(r, "Calls"))
        tot = float(_col(r, "TotalDurationNs"))
        e = out.setdefault(name, {"calls": 0, "total_ns": 0.0})
        e["calls"] += calls
        e["total_ns"] += tot
    for e in out.values():
        e["avg_ns"] = e["total_ns"] / max(e["calls"], 1)
    return out


def main_dispatch_durations(d):
    p = _find(os.path.join(d, "trace"), "*kernel_trace.csv")
    out = {}
    if not p:
        return out
    rows = defaultdict(list)
    for r in csv.DictReader(open(p)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        rows[short(r["Kernel_Name"])].append((g, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k, v in rows.items():
        gmax = max(g for g, _ in v)
        main = [t for g, t in v if 2 * g >= gmax]
        out[k] = {"main_calls": len(main), "main_avg_ns": sum(main) / len(main), "main_grid": gmax}
    return out


INFLATE = ("hbam::k_huff_tables", "hbam::k_inflate_huff", "hbam::k_inflate_huff<true>",
           "hbam::k_inflate_huff<false>", "hbam::k_inflate_lz77")


def inflate_stage_spans(d):
    """The inflate stage runs phase A (k_huff_tables + k_inflate_huff, pipeline
    stream) of chunk j+1 concurrently with phase B (k_inflate_lz77, second
    stream) of chunk j, so per-kernel durations overlap.  This groups maximal
    runs of inflate dispatches (by start time) and reports the wall span of the
    full-size runs: first phase-A start to last phase-B end of one pass."""
    p = _find(os.path.join(d, "trace"), "*kernel_trace.csv")
    if not p:
        return None
    ds = []
    for r in csv.DictReader(open(p)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        ds.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), g))
    ds.sort()
    runs, cur = [], []
    for dsp in ds:
        if dsp[2] in INFLATE:
            cur.append(dsp)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    if not runs:
        return None
    work = [sum(g for _, _, n, g in r if n == "hbam::k_inflate_lz77") for r in runs]
    wmax = max(work)
    main = [r for r, w in zip(runs, work) if 2 * w >= wmax]
    spans = [max(e for _, e, _, _ in r) - min(s_ for s_, _, _, _ in r) for r in main]
    return {"passes": len(main), "avg_span_ns": sum(spans) / len(spans),
            "lz77_launches_per_pass": sum(1 for _, _, n, _ in main[0] if n == "hbam::k_inflate_lz77")}


def base_name(k):
    """A kernel's name without its template arguments (k_inflate_huff<true>)."""
    return k.split("<")[0]


def counters(d, sub, merge_instances=False):
    """Per kernel: each counter averaged over its dispatches, and over its
    full-size ("main:") dispatches; main_dispatches = how many those are.
    merge_instances: template instances of a kernel count as one kernel."""
    p = _find(os.path.join(d, sub), "*counter_collection.csv")
    agg = defaultdict(lambda: defaultdict(list))
    if not p:
        return {}
    per_dispatch = defaultdict(float)
    names = {}
    grid = {}
    for r in csv.DictReader(open(p)):
        k = short(_col(r, "Kernel_Name", "KernelName"))
        if merge_instances:
            k = base_name(k)
        cn = _col(r, "Counter_Name", "CounterName")
        v = float(_col(r, "Counter_Value", "CounterValue"))
        disp = _col(r, "Dispatch_Id", "DispatchId", "Correlation_Id")
        per_dispatch[(k, cn, disp)] += v
        names[(k, cn, disp)] = (k, cn)
        grid[(k, cn, disp)] = int(_col(r, "Grid_Size"))
    gmax = defaultdict(int)
    for key, g in grid.items():
        gmax[names[key][0]] = max(gmax[names[key][0]], g)
    main_disp = defaultdict(set)
    for key, v in per_dispatch.items():
        k, cn = names[key]
        agg[k][cn].append(v)
        if 2 * grid[key] >= gmax[k]:
            agg[k]["main:" + cn].append(v)
            main_disp[k].add(key[2])
    out = {k: {cn: sum(vs) / len(vs) for cn, vs in cs.items()} for k, cs in agg.items()}
    for k, ds in main_disp.items():
        out[k]["main_dispatches"] = len(ds)
    return out


def totals(d, sub):
    """Per kernel (template instances merged): each counter summed over every
    dispatch of the run, and the dispatch count."""
    p = _find(os.path.join(d, sub), "*counter_collection.csv")
    out = defaultdict(lambda: defaultdict(float))
    if not p:
        return {}
    seen = defaultdict(set)
    for r in csv.DictReader(open(p)):
        k = base_name(short(_col(r, "Kernel_Name", "KernelName")))
        out[k][_col(r, "Counter_Name", "CounterName")] += float(_col(r, "Counter_Value", "CounterValue"))
        seen[k].add(_col(r, "Dispatch_Id", "DispatchId", "Correlation_Id"))
    for k, ds in seen.items():
        out[k]["dispatches"] = len(ds)
    return {k: dict(v) for k, v in out.items()}


def main():
    d = sys.argv[1]
    ks = kernel_stats(d)
    for k, e in main_dispatch_durations(d).items():
        ks.setdefault(k, {}).update(e)
    pm = {}
    for sub in ("fetch", "write", "sq"):
        for k, cs in counters(d, sub).items():
            pm.setdefault(k, {}).update(cs)
    res = {}
    for k in sorted(set(ks) | set(pm), key=lambda k: -ks.get(k, {}).get("total_ns", 0)):
        e = dict(ks.get(k, {}))
        c = pm.get(k, {})
        for pre in ("", "main:"):
            tag = pre.replace(":", "_")
            if pre + "FETCH_SIZE" in c:
                e[tag + "fetch_kb_raw"] = c[pre + "FETCH_SIZE"]
                e[tag + "fetch_bytes_corrected"] = c[pre + "FETCH_SIZE"] * 1024 * 2
            if pre + "WRITE_SIZE" in c:
                e[tag + "write_kb_raw"] = c[pre + "WRITE_SIZE"]
                e[tag + "write_bytes"] = c[pre + "WRITE_SIZE"] * 1024
        for cn, v in c.items():
            if cn.startswith("SQ_"):
                e[cn] = v
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_per_lds_inst"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"]
        if "SQ_LDS_IDX_ACTIVE" in c and c.get("SQ_INSTS_LDS"):
            e["lds_cycles_per_lds_inst"] = c["SQ_LDS_IDX_ACTIVE"] / c["SQ_INSTS_LDS"]
        for pre in ("", "main:"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; one LDS array per CU (256)
            if c.get(pre + "SQ_LDS_IDX_ACTIVE") is not None and c.get(pre + "GRBM_GUI_ACTIVE"):
                e[pre.replace(":", "_") + "lds_frac"] = c[pre + "SQ_LDS_IDX_ACTIVE"] / (256 * c[pre + "GRBM_GUI_ACTIVE"] / 8)
        if c.get("SQ_ACTIVE_INST_VALU") is not None and c.get("SQ_WAVE_CYCLES"):
            e["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        res[k] = e
    # every dispatch of the run summed (FETCH x 2, KiB -> B); bench.py's PMC
    # child decodes the split once, so there this is one pass's HBM traffic
    # (plus the few header-read dispatches of the open)
    tf, tw = totals(d, "fetch"), totals(d, "write")
    run_total = None
    if tf and tw:
        per = {k: {"fetch_bytes": tf.get(k, {}).get("FETCH_SIZE", 0) * 2048,
                   "write_bytes": tw.get(k, {}).get("WRITE_SIZE", 0) * 1024,
                   "dispatches": int(tf.get(k, {}).get("dispatches", 0))} for k in set(tf) | set(tw)}
        run_total = {"bytes": sum(v["fetch_bytes"] + v["write_bytes"] for v in per.values()),
                     "per_kernel": dict(sorted(per.items(), key=lambda kv: -(kv[1]["fetch_bytes"] +
                                                                           kv[1]["write_bytes"])))}
    print(json.dumps({"kernels": res, "inflate_stage": inflate_stage_spans(d), "pmc_run_total": run_total},
                     indent=1))


if __name__ == "__main__":
    main()
