#!/bin/bash
# r04o: BPLA exp path with three rows per lane (build/libsk_r3.so, -DSK_BPLA_ROWS=3):
# BPLA / async GPU tests on it, then C4 A/B against the two-row default, twice
set -o pipefail
TAG=${1:-r04o}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],3), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch parity', p.get('max_rel_err'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
SK_LIB_PATH=$PWD/build/libsk_r3.so timeout -k 10 400 python -u -m pytest tests/test_bpla.py tests/test_async.py tests/test_large_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_r3.log 2>&1 || { tail -30 $OUT/pytest_r3.log; exit 1; }
tail -1 $OUT/pytest_r3.log
run r3_1 SK_LIB_PATH=$PWD/build/libsk_r3.so python3 -u bench.py --config c4
run base_1 python3 -u bench.py --config c4 --no-cpu-baseline
run r3_2 SK_LIB_PATH=$PWD/build/libsk_r3.so python3 -u bench.py --config c4 --no-cpu-baseline
run base_2 python3 -u bench.py --config c4 --no-cpu-baseline
