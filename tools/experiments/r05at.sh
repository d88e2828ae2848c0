#!/bin/bash
# r05at: 4-D column kernel, positions with no stacking chain (most: bp is sparse) run a row loop without the stacking branches: stem4d GPU tests, C3 twice
set -o pipefail
OUT=gpurun_out/r05at; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
timeout -k 10 300 python -u -m pytest tests/test_stem4d.py tests/test_stem4d_col_schedule.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/c3_$r.log 2>&1 || { tail -20 $OUT/c3_$r.log; exit 1; }
  line $OUT/c3_$r.log "c3 $r"
done
