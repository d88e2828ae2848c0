#!/bin/bash
# r04u: C4 pairs per bench step (--slices 16 = 131k pairs, 8 = 262k, 4 = 525k); C3 at 512 pairs again
set -o pipefail
TAG=${1:-r04u}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],3))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run c4_s16a python3 -u bench.py --config c4 --no-cpu-baseline --slices 16
run c4_s8 python3 -u bench.py --config c4 --no-cpu-baseline --slices 8
run c4_s4 python3 -u bench.py --config c4 --no-cpu-baseline --slices 4
run c4_s16b python3 -u bench.py --config c4 --no-cpu-baseline --slices 16
run c3_default python3 -u bench.py --config c3 --no-cpu-baseline
