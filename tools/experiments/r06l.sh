#!/bin/bash
# r06l: the DAG kernel without its item-loop / per-pair spills (staging thread
# index and the gamma-sum lane opaque per item / pair, the pair counter from
# 0): MAXK 16 at 0 scratch bytes. Parity on the config-size fixtures, then NS
# and C5 A/B against the r06k tree, two rounds
set -o pipefail
OUT=gpurun_out/r06l; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab.sh r06l "ns c5" 2 build/libsk_base.so build/libsk_nospill.so
