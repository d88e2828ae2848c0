#!/bin/bash
# r06r: the whole NS Gram through sk_gram_sharded (bench --full) under the
# kernel trace, with the host planning times (SK_HOST_STATS): how much prep
# the product call exposes before its first stem launch
set -o pipefail
OUT=gpurun_out/r06r; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
SK_HOST_STATS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --full --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
grep "\[sk" $OUT/bench.log | tail -30
