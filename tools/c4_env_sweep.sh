#!/bin/bash
# C4 kernel time per launch for each environment setting given (one per
# argument, e.g. "SK_BPLA_IWAVES=4 SK_BPLA_CHUNK=2").  Usage: tools/c4_env_sweep.sh TAG SETTING...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/run_$i.log 2>&1 || { tail -20 $OUT/run_$i.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/run_$i.log').read().strip().splitlines()[-1]); r=l['roofline']; print('$setting:', round(l['value']), 'pairs/s', round(r['kernel_ms_per_launch'],3), 'ms/launch')"
done
