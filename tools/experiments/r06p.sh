#!/bin/bash
# r06p: the IY sweep's record fields by bit-field extracts and the g^k table
# base in an SGPR (36 -> 31 VALU per three chunks), with the chunk loop's exit
# test per chunk (swp0) or a uniform trip count (swp1, SK_SWEEP_TRIP=1: 19-21 -> 10-12
# SALU per three chunks), against the r06 final tree: parity of both, NS, C2
# and C5 A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06p; mkdir -p $OUT; export TMPDIR=/tmp
for v in swp0 swp1; do
  SK_LIB_PATH=$PWD/build/libsk_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_random_sweep.py tests/test_gpu_parity.py > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
bash tools/ab.sh r06p "ns c2 c5" 2 build/libsk_base.so build/libsk_swp0.so build/libsk_swp1.so
