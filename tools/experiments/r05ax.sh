#!/bin/bash
# r05ax: 4-D column kernel, rows fetched two steps ahead (SK4C_PF=2: every row step fetches in its tail) against one (default, direct fetch), C3 twice each
set -o pipefail
OUT=gpurun_out/r05ax; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/c3_$r.log 2>&1 || { tail -20 $OUT/c3_$r.log; exit 1; }
  line $OUT/c3_$r.log "c3 $r"
  SK_LIB_PATH=$PWD/build/libsk_pf2.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/pf2_$r.log 2>&1 || { tail -20 $OUT/pf2_$r.log; exit 1; }
  line $OUT/pf2_$r.log "pf2 $r"
done
