#!/bin/bash
# r06k: 12-wave register classes of 13, 14 and 15 slots (C2's y's, a tenth of
# NS) against MAXK 16 for all of them (SK_WIDE_MIN=16): parity on the
# config-size fixtures, then NS and C2 A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06k; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab.sh r06k "ns c2" 2 build/libsk_wide16.so build/libsk_wide13.so
