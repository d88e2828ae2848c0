#!/bin/bash
# Memory-latency counters of the stem kernel (GPU box): tools/pmc_lat.sh OUT "COUNTERS" [L N]
OUT=${1:-gpurun_out/pmc_lat}; SET=$2; L=${3:-200}; N=${4:-64}
mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
timeout -k 10 120 rocprofv3 --pmc $SET -d $ROOT/$OUT -o run --output-format csv -- python3 $ROOT/tools/probe_perf.py $L $N stem > $ROOT/$OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $ROOT/$OUT/run.log
python3 - "$ROOT/$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "stem_kernel" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()): print(k, v)
PY
