#!/bin/bash
# r06ab: C2 and C3 with asynchronous calls (--async) against synchronous, two rounds
set -o pipefail
OUT=gpurun_out/r06ab; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for c in c2 c3; do
    for m in sync async; do
      A=""; [ $m == async ] && A="--async"
      timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline $A > $OUT/${c}_${m}_$r.log 2>&1 || { tail -20 $OUT/${c}_${m}_$r.log; exit 1; }
      python3 -c "import json; l=json.loads(open('$OUT/${c}_${m}_$r.log').read().strip().splitlines()[-1]); print('$c $m r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],2), 'ms/step')"
    done
  done
done
