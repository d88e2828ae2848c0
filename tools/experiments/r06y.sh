#!/bin/bash
# r06y: NS with the costliest DAG class launched first (SK_CLASS_ORDER=1, the
# experiments build; NS: MAXK 16 first, then 17, then 20) against the size
# order (20, 17, 16), two rounds
set -o pipefail
OUT=gpurun_out/r06y; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for o in 0 1; do
    SK_LIB_PATH=$PWD/build/libstem_kernel_amd_exp.so SK_CLASS_ORDER=$o timeout -k 10 600 python3 -u bench.py --config ns --no-cpu-baseline > $OUT/ns_${o}_$r.log 2>&1 || { tail -20 $OUT/ns_${o}_$r.log; exit 1; }
    python3 -c "import json; l=json.loads(open('$OUT/ns_${o}_$r.log').read().strip().splitlines()[-1]); print('ns order=$o r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],1))"
  done
done
