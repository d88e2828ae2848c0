#!/bin/bash
# C4 kernel time per launch against the pairs a wave streams back to back
# (SK_BPLA_CHUNK).  Usage: tools/c4_chunk_sweep.sh TAG "2 4 6 8"
set -o pipefail
TAG=${1:-c4sweep}; VALS=${2:-"2 4 6 8"}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for c in $VALS; do
  SK_BPLA_CHUNK=$c timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/chunk_$c.log 2>&1 || { tail -20 $OUT/chunk_$c.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/chunk_$c.log').read().strip().splitlines()[-1]); r=l['roofline']; print('chunk $c', round(l['value']), 'pairs/s', round(r['kernel_ms_per_launch'],3), 'ms/launch')"
done
