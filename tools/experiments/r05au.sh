#!/bin/bash
# r05au: 4-D column kernel, which chain of a row step runs the wrap staging and fence wait:
# chain 1 (default build), 2 (st2) and 0 (st0, the r05ar kernel): stem4d GPU tests, C3 twice each
set -o pipefail
OUT=gpurun_out/r05au; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step')" $1 "$2"; }
timeout -k 10 300 python -u -m pytest tests/test_stem4d.py tests/test_stem4d_col_schedule.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/c3_$r.log 2>&1 || { tail -20 $OUT/c3_$r.log; exit 1; }
  line $OUT/c3_$r.log "ch1 $r"
  for v in st2 st0; do
    SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 3 > $OUT/${v}_$r.log 2>&1 || { tail -20 $OUT/${v}_$r.log; exit 1; }
    line $OUT/${v}_$r.log "$v $r"
  done
done
