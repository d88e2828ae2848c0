#!/bin/bash
# 4-D GPU tests, then C3 A/B: the column kernel (in-tree default) against the
# span kernels (SK4_NO_COL=1).  Usage: tools/gpu_c3.sh TAG
set -o pipefail
TAG=${1:-c3}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_async.py tests/test_stem4d.py tests/test_stem4d_long.py tests/test_large_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stem4d or async" > $OUT/pytest_4d.log 2>&1 || { tail -30 $OUT/pytest_4d.log; exit 1; }
tail -1 $OUT/pytest_4d.log
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'], 'parity', (l.get('parity') or {}).get('max_rel_err'))" $1 "$2"; }
timeout -k 10 300 python3 -u bench.py --config c3 > $OUT/c3_col.log 2>&1 || { tail -20 $OUT/c3_col.log; exit 1; }
line $OUT/c3_col.log "c3 col"
SK4_NO_COL=1 timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > $OUT/c3_pre.log 2>&1 || { tail -20 $OUT/c3_pre.log; exit 1; }
line $OUT/c3_pre.log "c3 pre"
timeout -k 10 400 python3 -u bench.py --config ns --no-cpu-baseline > $OUT/ns_async.log 2>&1 || { tail -20 $OUT/ns_async.log; exit 1; }
line $OUT/ns_async.log "ns async"
timeout -k 10 400 python3 -u bench.py --config ns --no-cpu-baseline --sync > $OUT/ns_sync.log 2>&1 || { tail -20 $OUT/ns_sync.log; exit 1; }
line $OUT/ns_sync.log "ns sync"
