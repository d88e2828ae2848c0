#!/usr/bin/env python3
"""Turn tools/pmc_bench.sh output into profiles/<kernel>_traffic.json.

HBM bytes of the dominant kernel's dispatches = 2 x FETCH_SIZE (gfx950
reports half the bytes of wide streaming reads, MI355X_MICROARCH.md) +
WRITE_SIZE, both in KiB per dispatch; divided by the algorithmic cells of
the bench step (read from the bench JSON line in the pass's log), giving HBM
bytes per cell, which bench.py multiplies back per launch.
Usage: tools/pmc_traffic.py OUTDIR KERNEL_SUBSTR KIND LENGTH OUT_JSON"""
import csv
import glob
import json
import os
import sys

out, ksub, kind, length, dst = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
tot = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = 0.0
    for f in glob.glob(os.path.join(out, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"] and r["Counter_Name"] == c:
                v += float(r["Counter_Value"])
    tot[c] = v * 1024.0
line = None
for ln in open(os.path.join(out, "FETCH_SIZE.log")):
    if ln.startswith("{") and '"metric"' in ln:
        line = json.loads(ln)
rf = line["roofline"]
launches = rf["launches"]
hbm = 2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]
# cells of the timed step: the bench reports algorithmic bytes; cells are
# recovered from sk_last_timing via the per-launch traffic model below
cells = line.get("cells_per_step")
res = {"kernel": kind, "length": length, "fetch_bytes_x2": 2.0 * tot["FETCH_SIZE"],
       "write_bytes": tot["WRITE_SIZE"], "hbm_bytes_step": hbm,
       "algorithmic_bytes_step": rf["algorithmic_per_launch"] * launches,
       "launches": launches, "cells_step": cells,
       "hbm_bytes_per_cell": hbm / cells if cells else None,
       "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE on bench.py --config "
                 f"{line['config']['workload'].split(':')[0]} --steps 1 --warmup 0"}
json.dump(res, open(dst, "w"), indent=1)
print(json.dumps(res, indent=1))
