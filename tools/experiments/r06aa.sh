#!/bin/bash
# r06aa: the MAXK 20 class (y of 1,088-1,279 nodes) on the 12-wave layout
# (halves, per-node f32 weights, no prefetched row): w20a with the edges in LDS
# and 128-node MATCH passes (the LDS fits 10 waves at NS), w20b with the edges
# from L2 and 64-node passes (12 waves); 172 / 136 scratch bytes against 0 at
# 8 waves.  Parity on the config-size fixtures, NS and C5 A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06aa; mkdir -p $OUT; export TMPDIR=/tmp
for v in w20a w20b; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
bash tools/ab.sh r06aa "ns c5" 2 build/libsk_base.so build/libsk_w20a.so build/libsk_w20b.so
