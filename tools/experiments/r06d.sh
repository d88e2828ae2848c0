#!/bin/bash
# r06d: DAG kernel phase A through LDS-DMA (SK_ADMA 1: the 12-wave MAXK 16 class, 2: every class):
# parity on the config-size fixtures, then NS A/B against SK_ADMA=0, two rounds
set -o pipefail
OUT=gpurun_out/r06d; mkdir -p $OUT; export TMPDIR=/tmp
for v in adma1 adma2; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gamma.py tests/test_gpu_parity.py > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
bash tools/ab.sh r06d "ns" 2 build/libsk_adma0.so build/libsk_adma1.so build/libsk_adma2.so
