#!/bin/bash
# r06 final tree (after the last source edits): GPU suite + smoke + NS
# measurement round trip, the driver's bench command, the other configs
set -o pipefail
bash tools/measure.sh ns r06zz_ns --tests || exit 1
OUT=gpurun_out/r06zz_ns; export TMPDIR=/tmp
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
tail -1 $OUT/bench_driver.log | cut -c1-160
for c in c2 c3 c4 c5; do
  bash tools/measure.sh $c r06zz_$c || exit 1
  tail -1 gpurun_out/r06zz_$c/bench.log | cut -c1-120
done
