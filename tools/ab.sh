#!/bin/bash
# A/B of library builds on bench configs: for each round, each config, each
# library (the in-tree build is "-"), one bench line (no CPU baseline).
# Usage: tools/ab.sh TAG "configs" ROUNDS lib...
set -o pipefail
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for r in $(seq $ROUNDS); do
  for c in $CFGS; do
    i=0
    for lib in "$@"; do
      i=$((i+1))
      L=""; [ "$lib" != "-" ] && L="$PWD/$lib"
      SK_LIB_PATH=$L timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline > $OUT/${c}_${i}_$r.log 2>&1 || { tail -20 $OUT/${c}_${i}_$r.log; exit 1; }
      python3 -c "import json; l=json.loads(open('$OUT/${c}_${i}_$r.log').read().strip().splitlines()[-1]); r=l['roofline']; print('$c $lib r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')"
    done
  done
done
