#!/usr/bin/env python3
"""Fold one tools/measure.sh run into profiles/<config>_traffic.json.

Inputs (OUTDIR from tools/measure.sh):
  prof/         rocprofv3 --kernel-trace --stats of bench.py (default steps)
  FETCH_SIZE/   rocprofv3 --pmc FETCH_SIZE   of bench.py --steps 1 --warmup 0
  WRITE_SIZE/   rocprofv3 --pmc WRITE_SIZE   (same command)
  LDS/          rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
                SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE (same command)
  *.log         the bench JSON lines of those runs

HBM bytes of the dominant kernel = 2 x FETCH_SIZE + WRITE_SIZE (gfx950:
FETCH_SIZE counts half the bytes of wide streaming reads; WRITE_SIZE is exact
for 16-B stores; MI355X_MICROARCH.md "HBM [CDNA4]"), divided by the
algorithmic cells of the counted step -> bytes per cell, which bench.py
scales back to its own launches.  The kernel trace gives the launches'
average duration (what the bench's HIP events must agree with) and their
overlap (sum of durations / union of intervals, per step), so

    frac = traffic_per_launch / (avg_launch_ns / overlap) / 8 TB/s

is recomputable from this file alone.  The LDS pass gives the binding
resource of the DAG kernel: LDS-array active cycles over the CU cycles of
the kernel, SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs).

Usage: tools/profile_summary.py OUTDIR CONFIG KERNEL_SUBSTR OUT_JSON"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stem_kernel_amd import provenance  # noqa: E402

PEAK = 8.0e12
KIND = {"ns": ("ss", 200), "c2": ("ss", 150), "c5": ("stem", 300), "c3": ("stem4d", 200), "c4": ("bpla", 210)}


def bench_line(path):
    line = None
    for ln in open(path):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    if line is None:
        raise SystemExit(f"no bench line in {path}")
    return line


def pmc(d, ksub):
    tot, disp = {}, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub not in r["Kernel_Name"]:
                continue
            disp.add((f, r.get("Dispatch_Id")))
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    tot["dispatches"] = len(disp)
    return tot


def trace(d, ksub, launches_per_step):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    durs = [e - s for s, e, _ in rows]
    # per step: the step's launches (in start order), union of their intervals
    spans, sums = [], []
    for k in range(0, len(rows) - launches_per_step + 1, launches_per_step):
        grp = rows[k:k + launches_per_step]
        iv = sorted((s, e) for s, e, _ in grp)
        u, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                u += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        u += ce - cs
        spans.append(u)
        sums.append(sum(e - s for s, e in iv))
    by_name = {}
    for s, e, n in rows:
        by_name.setdefault(n, []).append(e - s)
    return {"dispatches": len(rows), "avg_launch_ns": sum(durs) / max(1, len(durs)),
            "avg_launch_ns_timed": (sum(durs[launches_per_step:]) / max(1, len(durs) - launches_per_step)),
            "overlap": sum(sums[1:]) / max(1, sum(spans[1:])) if len(spans) > 1 else None,
            "span_ns_per_step_timed": sum(spans[1:]) / max(1, len(spans) - 1) if len(spans) > 1 else None,
            "per_kernel": {n: {"calls": len(v), "avg_ns": sum(v) / len(v)} for n, v in by_name.items()}}


def main():
    out, cfg, ksub, dst = sys.argv[1:5]
    kind, length = KIND[cfg]
    fl = bench_line(os.path.join(out, "FETCH_SIZE.log"))
    rf = fl["roofline"]
    launches = rf["launches"]
    cells = fl["cells_per_step"]
    f = pmc(os.path.join(out, "FETCH_SIZE"), ksub)
    w = pmc(os.path.join(out, "WRITE_SIZE"), ksub)
    hbm = 2.0 * f.get("FETCH_SIZE", 0.0) * 1024.0 + w.get("WRITE_SIZE", 0.0) * 1024.0
    res = {"kernel": kind, "config": cfg, "length": length, **provenance.stamp(),
           "kernel_substr": ksub,
           "fetch_bytes_x2": 2.0 * f.get("FETCH_SIZE", 0.0) * 1024.0,
           "write_bytes": w.get("WRITE_SIZE", 0.0) * 1024.0,
           "hbm_bytes_step": hbm, "launches_step": launches, "cells_step": cells,
           "hbm_bytes_per_cell": hbm / cells if cells else None,
           "hbm_bytes_per_launch": hbm / launches,
           "algorithmic_bytes_per_launch": rf["algorithmic_per_launch"],
           "pmc_dispatches": {"FETCH_SIZE": f["dispatches"], "WRITE_SIZE": w["dispatches"]},
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) -- bench.py --config {cfg} "
                     f"--steps 1 --warmup 0 --no-cpu-baseline; kernels matching '{ksub}'"}
    ldsd = os.path.join(out, "LDS")
    if os.path.isdir(ldsd):
        c = pmc(ldsd, ksub)
        ll = bench_line(os.path.join(out, "LDS.log"))
        cc = ll["cells_per_step"]
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        res["lds"] = {
            "counters": c,
            "lds_busy_frac": c["SQ_LDS_IDX_ACTIVE"] / (gui / 8.0 * 256.0) if gui else None,
            "bank_conflict_share": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
            if c.get("SQ_LDS_IDX_ACTIVE") else None,
            "valu_per_cell": c.get("SQ_INSTS_VALU", 0.0) * 64.0 / cc,
            "salu_per_cell": c.get("SQ_INSTS_SALU", 0.0) * 64.0 / cc,
            "lds_insts_per_cell": c.get("SQ_INSTS_LDS", 0.0) * 64.0 / cc,
            "cells_step": cc,
            "formula": "lds_busy_frac = SQ_LDS_IDX_ACTIVE (summed over CUs) / (GRBM_GUI_ACTIVE / 8 XCDs "
                       "x 256 CUs); per-cell counts are wave instructions x 64 / cells",
        }
    pd = os.path.join(out, "prof")
    if os.path.isdir(pd):
        bl = bench_line(os.path.join(out, "bench_prof.log"))
        lps = bl["roofline"]["launches"] // bl["steps"]
        t = trace(pd, ksub, lps)
        bpl = res["hbm_bytes_per_cell"] * bl["cells_per_step"] / lps if res["hbm_bytes_per_cell"] else None
        res["trace"] = dict(t, launches_per_step=lps, bench_kernel_ms_per_launch=bl["roofline"]
                            ["kernel_ms_per_launch"], bench_overlap=bl["roofline"]["overlap"])
        if bpl and t["overlap"]:
            eff = t["avg_launch_ns_timed"] / t["overlap"] * 1e-9
            res["trace"]["frac_from_trace"] = bpl / eff / PEAK
            res["trace"]["hbm_bytes_per_launch_bench_steps"] = bpl
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
