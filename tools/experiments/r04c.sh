#!/bin/bash
# r04c: C3 column kernel (LDS-only barriers) vs span kernels; C4 async vs sync;
# NS base / w12 / w12n alternating, async.
set -o pipefail
TAG=${1:-r04c}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', 'span/launch', round(r['effective_ms_per_launch'],3), r['kernel'], 'parity', p.get('max_rel_err'))" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 300 python -u -m pytest tests/test_stem4d.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pt4d.log 2>&1 || { tail -20 $OUT/pt4d.log; exit 1; }
tail -1 $OUT/pt4d.log
run c3_col python3 -u bench.py --config c3
run c4_async python3 -u bench.py --config c4 --no-cpu-baseline
run c4_sync python3 -u bench.py --config c4 --no-cpu-baseline --sync
for r in 1 2; do
  run ns_base_$r python3 -u bench.py --config ns --no-cpu-baseline
  run ns_w12_$r SK_LIB_PATH=$PWD/build/libsk_w12.so python3 -u bench.py --config ns --no-cpu-baseline
  run ns_w12n_$r SK_LIB_PATH=$PWD/build/libsk_w12n.so python3 -u bench.py --config ns --no-cpu-baseline
done
run ns_sync python3 -u bench.py --config ns --no-cpu-baseline --sync
