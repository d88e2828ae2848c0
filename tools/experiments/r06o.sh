#!/bin/bash
# r06o: the 12-wave MAXK 16 / 17 classes reading D's G1 in one pass (SK_M16_HALFD=0:
# no spill change) against halves: parity on the config-size fixtures, NS and C2 A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06o; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_halfd0.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab.sh r06o "ns c2" 2 build/libsk_base.so build/libsk_halfd0.so
