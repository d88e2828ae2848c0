#!/bin/bash
# r04t2: C3 pairs per bench step around 512 (--slices 1025 = 512, 820 = 640, 1367 = 384)
set -o pipefail
TAG=${1:-r04t2}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step frac', round(r['frac'],3))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run s1025a python3 -u bench.py --config c3 --no-cpu-baseline
run s820 python3 -u bench.py --config c3 --no-cpu-baseline --slices 820
run s1367 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1367
run s1025b python3 -u bench.py --config c3 --no-cpu-baseline
