#!/bin/bash
# r06i: three-row BPLA window without the column-1 selects (row C's left reset at the wrap):
# BPLA parity suite on it, then C4 A/B against the r06 tree's kernel, two rounds
set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_bpla1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bpla.py "tests/test_large_configs.py::test_bpla_c4_alignments" > $OUT/pytest_bpla1.log 2>&1 || { tail -20 $OUT/pytest_bpla1.log; exit 1; }
echo "bpla1: $(tail -1 $OUT/pytest_bpla1.log)"
bash tools/ab.sh r06i "c4" 2 build/libsk_bpla0.so build/libsk_bpla1.so
