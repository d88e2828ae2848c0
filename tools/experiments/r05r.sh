#!/bin/bash
# r05r: the product path end to end -- full NS Gram through sk_gram_sharded (bench --full), kernel trace
set -o pipefail
OUT=gpurun_out/r05r; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
  python3 -u $ROOT/bench.py --config ns --full --no-cpu-baseline > $OUT/full.log 2>&1 || { tail -20 $OUT/full.log; exit 1; }
tail -1 $OUT/full.log | cut -c1-600
