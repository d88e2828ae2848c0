#!/bin/bash
# r04t: C3 pairs per bench step (--slices 2050 = 256 pairs, 1025 = 512, 683 = 768)
set -o pipefail
TAG=${1:-r04t}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],3))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run s2050a python3 -u bench.py --config c3 --no-cpu-baseline
run s1025 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1025
run s683 python3 -u bench.py --config c3 --no-cpu-baseline --slices 683 --steps 3
run s2050b python3 -u bench.py --config c3 --no-cpu-baseline
