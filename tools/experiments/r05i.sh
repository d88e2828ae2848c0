#!/bin/bash
# r05i: 4-D GPU tests on the PF 1 / NB 4 default, then C3 step sizes
set -o pipefail
TAG=${1:-r05i}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_async.py tests/test_stem4d.py tests/test_stem4d_long.py tests/test_large_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stem4d or async" > $OUT/pytest_4d.log 2>&1 || { tail -30 $OUT/pytest_4d.log; exit 1; }
tail -1 $OUT/pytest_4d.log
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch', 'parity', (l.get('parity') or {}).get('max_rel_err'))" $1 "$2"; }
for s in ${SLICES:-1367 684 513 342}; do
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --slices $s --steps 3 --warmup 1 > $OUT/c3_$s.log 2>&1 || { tail -20 $OUT/c3_$s.log; exit 1; }
  line $OUT/c3_$s.log "c3 slices $s"
done
