#!/bin/bash
# bench lines of the given configs (no CPU baseline).  Usage: tools/quick_bench.sh TAG CONFIG...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  python3 -c "import json; l=json.loads(open('$OUT/$c.log').read().strip().splitlines()[-1]); r=l['roofline']; print('$c', round(l['value']), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r['frac'],4), r.get('basis','')[:40])"
done
