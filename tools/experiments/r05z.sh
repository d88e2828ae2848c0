#!/bin/bash
# r05z: fold kernel (diagonal-major tables, LDS ring): GPU fold tests, throughput, per-pass cycles
set -o pipefail
OUT=gpurun_out/r05z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fold.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_fold.log 2>&1 || { tail -30 $OUT/pytest_fold.log; exit 1; }
tail -1 $OUT/pytest_fold.log
timeout -k 10 300 python3 -u tools/fold_bench.py 4096 200 32 > $OUT/fold200.log 2>&1 || { tail -20 $OUT/fold200.log; exit 1; }
tail -1 $OUT/fold200.log
timeout -k 10 300 python3 -u tools/fold_bench.py 1024 400 8 > $OUT/fold400.log 2>&1 || { tail -20 $OUT/fold400.log; exit 1; }
tail -1 $OUT/fold400.log
SK_LIB_PATH=$PWD/build/libsk_ft.so timeout -k 10 300 python3 -u tools/fold_bench.py 1024 200 4 > $OUT/ft.log 2>&1 || { tail -20 $OUT/ft.log; exit 1; }
grep "^fold b" $OUT/ft.log | head -4
