#!/bin/bash
# Stall-reason counters of one config's dominant kernel (GPU box):
#   tools/pmc_stall.sh OUT CONFIG KSUB [ENV=VAL ...]
# WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) +
# ACTIVE_INST_ANY ~= WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots).
OUT=$1; CFG=$2; KSUB=$3; shift 3
mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
timeout -s KILL 300 env "$@" rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES -d $ROOT/$OUT -o run --output-format csv -- \
  python3 $ROOT/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $ROOT/$OUT/run.log 2>&1 || { tail -5 $ROOT/$OUT/run.log; exit 1; }
python3 - "$ROOT/$OUT" "$KSUB" <<'PY'
import csv, glob, sys, collections, json
tot = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
wc = tot.get("SQ_WAVE_CYCLES", 0) or 1
res = {k: v for k, v in sorted(tot.items())}
res["share"] = {k: tot[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                          "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS")}
json.dump(res, open(sys.argv[1] + "/stall.json", "w"), indent=1)
print(sys.argv[2], json.dumps(res["share"]))
PY
