#!/bin/bash
# r06ad: C3 steps of 2,042 pairs (slices 257) against 1,023 (513), two rounds
set -o pipefail
OUT=gpurun_out/r06ad; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for s in 513 257; do
    timeout -k 10 600 python3 -u bench.py --config c3 --no-cpu-baseline --slices $s > $OUT/c3_${s}_$r.log 2>&1 || { tail -20 $OUT/c3_${s}_$r.log; exit 1; }
    python3 -c "import json; l=json.loads(open('$OUT/c3_${s}_$r.log').read().strip().splitlines()[-1]); print('c3 1/$s r$r', round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')"
  done
done
