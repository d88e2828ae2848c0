#!/bin/bash
# r04k: final-tree check -- full GPU suite + smoke, every config's bench line, NS host timings
set -o pipefail
TAG=${1:-r04k}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; c=l['config']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],3), 'stale', r.get('stale'), 'parity', p.get('max_rel_err'), {k: v['max_rel_err'] for k, v in (p.get('components') or {}).items()}, 'build', c.get('host_build_s'), 'upload', c.get('upload_s'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run ns SK_HOST_STATS=1 python3 -u bench.py --config ns
grep "\[sk" $OUT/ns.log | head -12
run c4 python3 -u bench.py --config c4 --no-cpu-baseline
run c3 python3 -u bench.py --config c3 --no-cpu-baseline
run c3_prold SK_LIB_PATH=$PWD/build/libsk_prold.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_b python3 -u bench.py --config c3 --no-cpu-baseline
run c2 python3 -u bench.py --config c2 --no-cpu-baseline
run c5 python3 -u bench.py --config c5 --no-cpu-baseline
# column kernel: full-barrier interval F (SK4C_F) sweep
run c3col_f8 SK4_COL=1 python3 -u bench.py --config c3 --no-cpu-baseline
run c3col_old SK4_COL=1 SK_LIB_PATH=$PWD/build/libsk_prold.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3col_f16 SK4_COL=1 SK4C_F=16 python3 -u bench.py --config c3 --no-cpu-baseline
run c3col_f32 SK4_COL=1 SK4C_F=32 python3 -u bench.py --config c3 --no-cpu-baseline
# C4 kernel trace: gaps between consecutive BPLA launches (uploads on the copy stream)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline > $OUT/prof_c4.log 2>&1 || { tail -20 $OUT/prof_c4.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof_c4/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "bpla_fast_items" in r["Kernel_Name"]]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
print("C4 items-kernel gaps us:", [round(g, 1) for g in gaps])
PY
