#!/bin/bash
# r06q: NS with asynchronous calls (--async: step t+1 planned while step t
# runs, no host gap between steps) against synchronous, two rounds; C5 too
set -o pipefail
OUT=gpurun_out/r06q; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for c in ns c5; do
    for m in sync async; do
      A=""; [ $m == async ] && A="--async"
      timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline $A > $OUT/${c}_${m}_$r.log 2>&1 || { tail -20 $OUT/${c}_${m}_$r.log; exit 1; }
      python3 -c "import json; l=json.loads(open('$OUT/${c}_${m}_$r.log').read().strip().splitlines()[-1]); r=l['roofline']; print('$c $m r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],2), 'ms/step frac', round(r['frac'],4), 'eff', round(r['effective_ms_per_launch'],1))"
    done
  done
done
