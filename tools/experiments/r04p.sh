#!/bin/bash
# r04p: C4 chunk size (pairs a wave streams back to back, SK_BPLA_CHUNK) with three rows per lane
set -o pipefail
TAG=${1:-r04p}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
B="python3 -u bench.py --config c4 --no-cpu-baseline"
for c in 8 4 6 10 12 16 8; do run chunk$c SK_BPLA_CHUNK=$c $B; done
