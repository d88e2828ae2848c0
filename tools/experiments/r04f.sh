#!/bin/bash
# r04f: 4-D pre-combined span kernel at 4 waves per SIMD (SK4P_WPE=4, with and without the 2-row prefetch), A/B/C twice
set -o pipefail
TAG=${1:-r04f}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch', r['kernel'])" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
timeout -k 10 400 python -u -m pytest tests/test_stem4d.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_s4.log 2>&1 || { tail -30 $OUT/pytest_s4.log; exit 1; }
tail -1 $OUT/pytest_s4.log
for r in 1 2; do
run c3_pre_$r python3 -u bench.py --config c3 --no-cpu-baseline
run c3_p4_$r SK_LIB_PATH=$PWD/build/libsk_c3p4.so python3 -u bench.py --config c3 --no-cpu-baseline
run c3_p4pf1_$r SK_LIB_PATH=$PWD/build/libsk_c3p4pf1.so python3 -u bench.py --config c3 --no-cpu-baseline
done
