#!/bin/bash
# r05a: column-group 4-D kernel (NB chains per position): GPU parity of the
# 4-D tests, then C3 with 512- and 384-pair steps, and the span kernel beside it
set -o pipefail
TAG=${1:-r05a}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch frac', round(r.get('frac') or 0,3), 'par', l.get('parity',{}).get('max_rel_err'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_stem4d.py tests/test_stem4d_long.py \
  tests/test_large_configs.py -k "stem4d" -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run c3_col512 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1025 --steps 3 --warmup 1
run c3_col384 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1367 --steps 3 --warmup 1
run c3_span384 SK4_SPAN=1 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1367 --steps 3 --warmup 1
