#!/bin/bash
# r05y: McCaskill fold throughput (tools/fold_bench.py) and per-pass cycles (SK_FOLD_TIMING build)
set -o pipefail
OUT=gpurun_out/r05y; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/fold_bench.py 4096 200 32 > $OUT/fold.log 2>&1 || { tail -20 $OUT/fold.log; exit 1; }
tail -1 $OUT/fold.log
SK_LIB_PATH=$PWD/build/libsk_ft.so timeout -k 10 300 python3 -u tools/fold_bench.py 1024 200 4 > $OUT/ft.log 2>&1 || { tail -20 $OUT/ft.log; exit 1; }
grep "^fold b" $OUT/ft.log | head -6
