#!/bin/bash
# r06 final tree: GPU suite + smoke + NS measurement round trip (tools/measure.sh:
# kernel trace, FETCH_SIZE / WRITE_SIZE / LDS passes, bench line), then one
# bench line per other config and the NS host pack timing (SK_HOST_STATS)
set -o pipefail
bash tools/measure.sh ns r06f_ns --tests || exit 1
OUT=gpurun_out/r06f_ns; export TMPDIR=/tmp
for c in c2 c3 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log
done
SK_HOST_STATS=1 timeout -k 10 400 python3 -u bench.py --config ns --steps 1 --warmup 0 --no-cpu-baseline > $OUT/host_stats.log 2>&1 || { tail -20 $OUT/host_stats.log; exit 1; }
grep "sk pack\|sk\]" $OUT/host_stats.log | head -20
