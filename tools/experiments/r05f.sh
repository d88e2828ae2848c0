#!/bin/bash
# r05f: 4-D column kernel builds: rows ahead (PF) x columns per group (NB),
# C3 at 768-pair steps, two rounds alternating on one box
set -o pipefail
TAG=${1:-r05f}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
line() { python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=l['roofline']; print(sys.argv[2], round(l['value'],1), 'pairs/s', round(l['ms_per_step'],1), 'ms/step', round(r['kernel_ms_per_launch'],2), 'ms/launch')" $1 "$2"; }
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  line $OUT/$name.log "$name"
}
for r in 1 2; do
  run pf4nb2_$r python3 -u bench.py --config c3 --no-cpu-baseline --slices 684 --steps 2 --warmup 1
  for v in pf3nb2 pf2nb3 pf2nb2; do
    run ${v}_$r SK_LIB_PATH=$PWD/build/libsk_$v.so python3 -u bench.py --config c3 --no-cpu-baseline --slices 684 --steps 2 --warmup 1
  done
done
