#!/usr/bin/env python3
"""Copy one tools/measure.sh run (gpurun_out/<run>) into profiles/<tag>_*:
the bench line, rocprofv3 kernel stats, the engine's kernel-trace rows, the
engine's rows of each counter pass and the folded traffic JSON -- everything
the bench line's roofline is recomputed from.
Usage: tools/archive.py gpurun_out/RUN TAG"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(src, dst, keep):
    with open(src) as f, open(dst, "w", newline="") as g:
        r = csv.DictReader(f)
        w = csv.DictWriter(g, fieldnames=r.fieldnames)
        w.writeheader()
        for row in r:
            if keep(row):
                w.writerow(row)


def main():
    run, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    sk = lambda row: "sk::" in row.get("Kernel_Name", "") or "sk_" in row.get("Kernel_Name", "")
    for ln in open(os.path.join(run, "bench.log")):
        if ln.startswith("{"):
            line = json.loads(ln)
    json.dump(line, open(os.path.join(prof, f"{tag}_bench.json"), "w"), indent=1)
    for f in glob.glob(os.path.join(run, "prof", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    for f in glob.glob(os.path.join(run, "prof", "**", "*kernel_trace.csv"), recursive=True):
        rows(f, os.path.join(prof, f"{tag}_kernel_trace.csv"), sk)
    for name in ("FETCH_SIZE", "WRITE_SIZE", "LDS"):
        for f in glob.glob(os.path.join(run, name, "**", "*counter_collection.csv"), recursive=True):
            rows(f, os.path.join(prof, f"{tag}_pmc_{name.lower()}.csv"), sk)
    for f in glob.glob(os.path.join(run, "*_traffic.json")):
        cfg = json.load(open(f))["config"]
        shutil.copy(f, os.path.join(prof, f"{cfg}_traffic.json"))
        shutil.copy(f, os.path.join(prof, f"{tag}_traffic.json"))
    print("archived", tag)


if __name__ == "__main__":
    main()
