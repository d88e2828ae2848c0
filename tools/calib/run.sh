#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (see fetch_calib.hip).
set -o pipefail
OUT=gpurun_out/calib; mkdir -p $OUT; export TMPDIR=/tmp
ROOT=$(pwd)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d $ROOT/$OUT/$c -o run --output-format csv -- $ROOT/tools/calib/fetch_calib > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
done
# kernel durations (reread_2 faster than reread_1: the second pass hits the Infinity Cache)
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/trace -o run --output-format csv -- $ROOT/tools/calib/fetch_calib > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c:
                kb = float(r["Counter_Value"])
                name = r["Kernel_Name"].split("(")[0]
                ref = 2**26 if "reread" in name else 2**30
                print(c, name, "KiB", kb, "ratio to", "64 MiB" if ref == 2**26 else "1 GiB", kb * 1024 / ref)
for f in glob.glob("gpurun_out/calib/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("TRACE", r["Kernel_Name"].split("(")[0], "ns", int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
PY
