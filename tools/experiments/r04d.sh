#!/bin/bash
# r04d: full GPU suite + smoke on the new defaults; C3 column variants; NS line.
set -o pipefail
TAG=${1:-r04d}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', 'span/launch', round(r['effective_ms_per_launch'],3), r['kernel'], 'parity', p.get('max_rel_err'), {k: v['max_rel_err'] for k, v in (p.get('components') or {}).items()})" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run c3_col python3 -u bench.py --config c3 --no-cpu-baseline
run c3_pf1 SK_LIB_PATH=$PWD/build/libsk_c3pf1.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_w16 SK_LIB_PATH=$PWD/build/libsk_c3w16.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_pre SK4_NO_COL=1 python3 -u bench.py --config c3 --no-cpu-baseline
run ns python3 -u bench.py --config ns
