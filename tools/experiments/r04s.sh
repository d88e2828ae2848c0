#!/bin/bash
# r04s: DAG kernel rows prefetched per row in the MAXK 20 (SK_NPF20) and MAXK <= 12 (SK_NPF12) classes: NS and C2, A/B/A
set -o pipefail
TAG=${1:-r04s}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
N="python3 -u bench.py --config ns --no-cpu-baseline --steps 4"
C="python3 -u bench.py --config c2 --no-cpu-baseline"
run ns_base1 $N
run ns_npf20_1 SK_LIB_PATH=$PWD/build/libsk_npf20a.so $N
run ns_base2 $N
run c2_base1 $C
run c2_npf12_1 SK_LIB_PATH=$PWD/build/libsk_npf12a.so $C
run c2_base2 $C
