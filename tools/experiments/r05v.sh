#!/bin/bash
# r05v: C3 A/B of 4-D column kernel builds (VARIANTS: build/libsk_<v>.so; "main" = in-tree), two rounds
set -o pipefail
TAG=${1:-r05v}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch')" $1 "$2"; }
for r in 1 2; do
  for v in ${VARIANTS:-main}; do
    if [ $v == main ]; then lib=""; else lib=$PWD/build/libsk_$v.so; fi
    SK_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/${v}_$r.log 2>&1 || { tail -20 $OUT/${v}_$r.log; exit 1; }
    line $OUT/${v}_$r.log "${v}_$r"
  done
done
