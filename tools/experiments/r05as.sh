#!/bin/bash
# r05as: 4-D column kernel, what the per-step barrier costs: C3 with s_barrier removed (nb: a timing probe, wrong values)
set -o pipefail
OUT=gpurun_out/r05as; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/c3_$r.log 2>&1 || { tail -20 $OUT/c3_$r.log; exit 1; }
  line $OUT/c3_$r.log "c3 $r"
  SK_LIB_PATH=$PWD/build/libsk_nb.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/nb_$r.log 2>&1 || { tail -20 $OUT/nb_$r.log; exit 1; }
  line $OUT/nb_$r.log "nb $r"
done
