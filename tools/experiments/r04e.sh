#!/bin/bash
# r04e: 4-D column kernel -- point-to-point wave sync (default) vs lockstep, link depth, W16
set -o pipefail
TAG=${1:-r04e}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'], 'parity', p.get('max_rel_err'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python -u -m pytest tests/test_stem4d.py tests/test_cpp_compat.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_s4.log 2>&1 || { tail -30 $OUT/pytest_s4.log; exit 1; }
tail -1 $OUT/pytest_s4.log
run c3_p2p python3 -u bench.py --config c3 --no-cpu-baseline
run c3_ls SK_LIB_PATH=$PWD/build/libsk_c3ls.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_d2 SK_LIB_PATH=$PWD/build/libsk_c3d2.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_w16 SK_LIB_PATH=$PWD/build/libsk_c3w16.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_pre SK4_NO_COL=1 python3 -u bench.py --config c3 --no-cpu-baseline
