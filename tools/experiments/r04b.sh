#!/bin/bash
# r04: C3 column kernel vs span kernels; NS async vs sync; NS MAXK16 at 12 waves.
set -o pipefail
TAG=${1:-r04b}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; p=l.get('parity') or {}; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'], 'frac', round(r['frac'],3), 'parity', p.get('max_rel_err'), {k: v['max_rel_err'] for k, v in (p.get('components') or {}).items()})" $1 "$2"; }
run() {  # name, env, args
  local name=$1; shift
  timeout -k 10 400 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
run c3_col python3 -u bench.py --config c3
run c3_pre SK4_NO_COL=1 python3 -u bench.py --config c3 --no-cpu-baseline
run ns_async python3 -u bench.py --config ns
run ns_sync python3 -u bench.py --config ns --no-cpu-baseline --sync
run ns_w12 SK_LIB_PATH=$PWD/build/libsk_w12.so python3 -u bench.py --config ns --no-cpu-baseline
run ns_w12n SK_LIB_PATH=$PWD/build/libsk_w12n.so python3 -u bench.py --config ns --no-cpu-baseline
run c2 python3 -u bench.py --config c2 --no-cpu-baseline
