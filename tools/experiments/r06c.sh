#!/bin/bash
# r06c: DAG kernel prefetch-queue variants: parity on the config-size fixtures
# for each library, then NS bench A/B (tools/ab.sh), one round
set -o pipefail
OUT=gpurun_out/r06c; mkdir -p $OUT; export TMPDIR=/tmp
for v in m16w8 m16w8q2 pfqdef; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gamma.py > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
bash tools/ab.sh r06c "ns" 1 build/libsk_pfq0.so build/libsk_m16w8.so build/libsk_m16w8q2.so build/libsk_pfqdef.so
