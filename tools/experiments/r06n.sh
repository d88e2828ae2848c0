#!/bin/bash
# r06n: sweep dummies on the free slot of their host-chosen banks (SK_DUMMY_BANK)
# against dummies spread by lane: parity on the config-size fixtures, NS, C2
# and C5 A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab.sh r06n "ns c2 c5" 2 build/libsk_base.so build/libsk_dbank.so
