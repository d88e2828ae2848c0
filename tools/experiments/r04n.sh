#!/bin/bash
# r04n: NS knobs re-swept at 12 waves per CU for MAXK 16: MATCH edge rounds (SK_MU),
# pass width (SK_PW), quad sums (SK_SEGSUM), work-item sizing (SK_GSS_K); base twice
set -o pipefail
TAG=${1:-r04n}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_launch'],3), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
B="python3 -u bench.py --config ns --no-cpu-baseline --steps 4"
run base1 $B
run mu2 SK_LIB_PATH=$PWD/build/libsk_mu2.so $B
run mu4 SK_LIB_PATH=$PWD/build/libsk_mu4.so $B
run pw2 SK_LIB_PATH=$PWD/build/libsk_pw2.so $B
run pw4 SK_LIB_PATH=$PWD/build/libsk_pw4.so $B
run seg0 SK_LIB_PATH=$PWD/build/libsk_seg0.so $B
run gss1 SK_GSS_K=1.0 $B
run gss2 SK_GSS_K=2.0 $B
run base2 $B
