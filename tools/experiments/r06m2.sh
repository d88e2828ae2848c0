#!/bin/bash
# r06m2: the spill fixes of r06l in the MAXK 16 class only (0 scratch bytes
# there; every other class as before): parity on the config-size fixtures,
# NS and C2 (all MAXK 16) A/B against the r06k tree, two rounds
set -o pipefail
OUT=gpurun_out/r06m2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab.sh r06m2 "ns c2" 2 build/libsk_base.so build/libsk_nospill16.so
