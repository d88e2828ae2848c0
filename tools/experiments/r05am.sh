#!/bin/bash
# r05am: 4-D column kernel step-part cycles (SK4C_TIMING build) on the r05al tree, C3 one step
set -o pipefail
OUT=gpurun_out/r05am; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_tm.so timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 1 --warmup 0 > $OUT/tm.log 2>&1 || { tail -20 $OUT/tm.log; exit 1; }
grep sk4c $OUT/tm.log | head -40
