#!/bin/bash
# r06ac: MATCH edge rounds of 2 or 4 x 64 edges (SK_MU) against 3, NS, two rounds
set -o pipefail
OUT=gpurun_out/r06ac; mkdir -p $OUT; export TMPDIR=/tmp
for v in mu2 mu4; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
bash tools/ab.sh r06ac "ns" 2 build/libsk_base.so build/libsk_mu2.so build/libsk_mu4.so
