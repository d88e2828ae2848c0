#!/bin/bash
# r04v: C4 pairs per bench step, larger: --slices 4 (a quarter of the Gram), 2, 1 (the whole Gram)
set -o pipefail
TAG=${1:-r04v}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],3), 'pairs/step', l['config'].get('pairs_per_step_per_gpu'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run c4_s4a python3 -u bench.py --config c4 --no-cpu-baseline --slices 4
run c4_s2 python3 -u bench.py --config c4 --no-cpu-baseline --slices 2
run c4_s1 python3 -u bench.py --config c4 --no-cpu-baseline --slices 1
run c4_s4b python3 -u bench.py --config c4 --no-cpu-baseline --slices 4
