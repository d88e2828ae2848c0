#!/bin/bash
# r06x: NS work-item sizing (SK_GSS_K, the experiments build) at the 1/8-Gram
# async steps: K = 1.5 (shipped) against 1.0 and 2.5, two rounds
set -o pipefail
OUT=gpurun_out/r06x; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for k in 1.5 1.0 2.5; do
    SK_LIB_PATH=$PWD/build/libstem_kernel_amd_exp.so SK_GSS_K=$k timeout -k 10 600 python3 -u bench.py --config ns --no-cpu-baseline > $OUT/ns_${k}_$r.log 2>&1 || { tail -20 $OUT/ns_${k}_$r.log; exit 1; }
    python3 -c "import json; l=json.loads(open('$OUT/ns_${k}_$r.log').read().strip().splitlines()[-1]); print('ns K=$k r$r', round(l['value']), 'pairs/s', round(l['ms_per_step'],1))"
  done
done
