#!/bin/bash
# Quick bench lines (no tests, no profiles) for the configs given:
#   tools/gpu_quick.sh ns c5 c2 ...   -> gpurun_out/quick_<cfg>.log
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline > gpurun_out/quick_$c.log 2>&1 || { tail -20 gpurun_out/quick_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/quick_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['value']), 'frac', round(d['roofline']['frac'],4), 'ms/launch', round(d['roofline']['kernel_ms_per_launch'],2), 'ms/step', round(d['ms_per_step'],1))"
done
