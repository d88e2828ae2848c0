#!/bin/bash
# r04w2: C5 pairs per bench step (--slices 128 = 262k pairs, 64 = 525k)
set -o pipefail
TAG=${1:-r04w2}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],3))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run c5_s128a python3 -u bench.py --config c5 --no-cpu-baseline
run c5_s64 python3 -u bench.py --config c5 --no-cpu-baseline --slices 64
run c5_s32 python3 -u bench.py --config c5 --no-cpu-baseline --slices 32
run c5_s128b python3 -u bench.py --config c5 --no-cpu-baseline
