#!/bin/bash
# r05ad: NS work-item sizing (SK_GSS_K) at the 1/16-Gram steps, two rounds
set -o pipefail
OUT=gpurun_out/r05ad; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
for r in 1 2; do
  for k in 1.5 1.0 1.25 2.0; do
    SK_GSS_K=$k timeout -k 10 300 python3 -u bench.py --config ns --no-cpu-baseline --steps 3 > $OUT/k${k}_$r.log 2>&1 || { tail -20 $OUT/k${k}_$r.log; exit 1; }
    line $OUT/k${k}_$r.log "K $k round $r"
  done
done
