#!/bin/bash
# r04j: BPLA call inputs in one H2D copy: tests, C4 twice, kernel trace (inter-launch gaps)
set -o pipefail
TAG=${1:-r04j}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'])" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python -u -m pytest tests/test_bpla.py tests/test_async.py tests/test_bpla_grad.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run c4_1 python3 -u bench.py --config c4 --no-cpu-baseline
run c4_2 python3 -u bench.py --config c4 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "bpla_fast_items" in r["Kernel_Name"]]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
print("items-kernel gaps us:", [round(g, 1) for g in gaps])
print("all kernels between:", sum(1 for r in rows if int(r["Start_Timestamp"]) > int(ks[1]["End_Timestamp"]) and int(r["End_Timestamp"]) < int(ks[2]["Start_Timestamp"])))
PY
