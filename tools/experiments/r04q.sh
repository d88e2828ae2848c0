#!/bin/bash
# r04q: C4 item size (pairs of one y per work item, SK_BPLA_ITEM) with three rows per lane
set -o pipefail
TAG=${1:-r04q}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
B="python3 -u bench.py --config c4 --no-cpu-baseline"
run item192a $B
for it in 96 288 384 576; do run item$it SK_BPLA_ITEM=$it $B; done
run item192b $B
