#!/bin/bash
# r05b: column-group 4-D kernel with rows 4 ahead and no full barriers:
# 4-D GPU parity, then C3 at 512-pair steps (and 768), and W = 6 beside it
set -o pipefail
TAG=${1:-r05b}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch frac', round(r.get('frac') or 0,3), 'par', (l.get('parity') or {}).get('max_rel_err'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_stem4d.py tests/test_stem4d_long.py \
  tests/test_large_configs.py -k "stem4d" -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run c3_col512 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1025 --steps 3 --warmup 1
run c3_col512_w6 SK4C_W=6 python3 -u bench.py --config c3 --no-cpu-baseline --slices 1025 --steps 3 --warmup 1
run c3_col768 python3 -u bench.py --config c3 --slices 684 --steps 2 --warmup 1 --cpu-pairs 8
