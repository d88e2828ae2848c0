#!/bin/bash
# r05m: last-wave split (no dropped wrap stores), shared y tables by row width: C3 A/B + step-part cycles
set -o pipefail
TAG=${1:-r05m}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch', 'parity', (l.get('parity') or {}).get('max_rel_err'))" $1 "$2"; }
timeout -k 10 300 python3 -u bench.py --config c3 --steps 2 --warmup 1 > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
line $OUT/c3.log "c3 share<=2"
for v in sh0 sh4; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  line $OUT/$v.log "c3 $v"
done
SK_LIB_PATH=$PWD/build/libsk_tm.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 1 --warmup 0 > $OUT/tm.log 2>&1 || { tail -20 $OUT/tm.log; exit 1; }
grep sk4c $OUT/tm.log | sort | head -8
