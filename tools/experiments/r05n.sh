#!/bin/bash
# r05n: column kernel variants: 4-D tests, C3, step-part cycles
set -o pipefail
TAG=${1:-r05n}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_stem4d.py tests/test_large_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stem4d" > $OUT/pytest_4d.log 2>&1 || { tail -30 $OUT/pytest_4d.log; exit 1; }
tail -1 $OUT/pytest_4d.log
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch', 'parity', (l.get('parity') or {}).get('max_rel_err'))" $1 "$2"; }
timeout -k 10 300 python3 -u bench.py --config c3 --steps 2 --warmup 1 > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
line $OUT/c3.log "c3"
SK_LIB_PATH=$PWD/build/libsk_tm.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 1 --warmup 0 > $OUT/tm.log 2>&1 || { tail -20 $OUT/tm.log; exit 1; }
line $OUT/tm.log "c3 timing build"
grep sk4c $OUT/tm.log | sort | head -8
