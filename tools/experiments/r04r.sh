#!/bin/bash
# r04r: BPLA launch tail -- the last round's items split in two (default) vs not (SK_BPLA_TAIL=0)
set -o pipefail
TAG=${1:-r04r}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python -u -m pytest tests/test_bpla.py tests/test_async.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python3 -u bench.py --config c4 --no-cpu-baseline"
run tail_1 $B
run notail_1 SK_BPLA_TAIL=0 $B
run tail_2 $B
run notail_2 SK_BPLA_TAIL=0 $B
