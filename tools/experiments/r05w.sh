#!/bin/bash
# r05w: NS step size (slices of the Gram per step): 48 (current) / 24 / 16
set -o pipefail
OUT=gpurun_out/r05w; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch')" $1 "$2"; }
for s in 48 24 16 48 24 16; do
  timeout -k 10 300 python3 -u bench.py --config ns --no-cpu-baseline --slices $s > $OUT/ns_$s.log 2>&1 || { tail -20 $OUT/ns_$s.log; exit 1; }
  line $OUT/ns_$s.log "ns slices $s"
done
