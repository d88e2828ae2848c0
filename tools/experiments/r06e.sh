#!/bin/bash
# r06e: a MAXK 17 register class (y of 1,025-1,088 non-leaf nodes, 12 waves like MAXK 16)
# against none (those y in the 8-wave MAXK 20 class): parity, then NS A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06e; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_k17.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gamma.py tests/test_gpu_parity.py > $OUT/pytest_k17.log 2>&1 || { tail -20 $OUT/pytest_k17.log; exit 1; }
echo "k17: $(tail -1 $OUT/pytest_k17.log)"
bash tools/ab.sh r06e "ns" 2 build/libsk_k17off.so build/libsk_k17.so
