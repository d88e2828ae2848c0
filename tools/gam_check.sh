#!/bin/bash
# gamma-row check: stem parity tests, then NS with and without gamma rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_golden.py tests/test_big_dag.py tests/test_large_configs.py \
  > gpurun_out/gam_tests.log 2>&1 || { tail -40 gpurun_out/gam_tests.log; exit 1; }
tail -3 gpurun_out/gam_tests.log
bash tools/gpu_quick.sh ns || exit 1
SK_NO_GAMMA=1 bash tools/gpu_quick.sh ns
