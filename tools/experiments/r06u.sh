#!/bin/bash
# r06u: NS bench steps of 1/8 of the Gram against 1/16 (async steps), two rounds
set -o pipefail
OUT=gpurun_out/r06u; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for s in 16 8; do
    timeout -k 10 600 python3 -u bench.py --config ns --no-cpu-baseline --slices $s > $OUT/ns_${s}_$r.log 2>&1 || { tail -20 $OUT/ns_${s}_$r.log; exit 1; }
    python3 -c "import json; l=json.loads(open('$OUT/ns_${s}_$r.log').read().strip().splitlines()[-1]); print('ns 1/$s r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(l['roofline']['frac'],4))"
  done
done
