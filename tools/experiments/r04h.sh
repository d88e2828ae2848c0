#!/bin/bash
# r04h: BPLA window hand-off through an LDS add (no read round trip): tests + C4 twice
set -o pipefail
TAG=${1:-r04h}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'])" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python -u -m pytest tests/test_bpla.py tests/test_async.py tests/test_large_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run c4_1 python3 -u bench.py --config c4 --no-cpu-baseline
run c4_2 python3 -u bench.py --config c4 --no-cpu-baseline
