#!/bin/bash
# r05aw: 4-D column kernel, does the row fetch latency matter: C3 with every direct fetch reading row 1 (L2-resident; l2f: a timing probe, wrong values)
set -o pipefail
OUT=gpurun_out/r05aw; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/c3_$r.log 2>&1 || { tail -20 $OUT/c3_$r.log; exit 1; }
  line $OUT/c3_$r.log "c3 $r"
  SK_LIB_PATH=$PWD/build/libsk_l2f.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/l2f_$r.log 2>&1 || { tail -20 $OUT/l2f_$r.log; exit 1; }
  line $OUT/l2f_$r.log "l2f $r"
done
