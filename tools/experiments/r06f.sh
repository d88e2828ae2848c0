#!/bin/bash
# r06f: IY sweep without the dummy select (dummy records on the class's free last slot; every
# register class keeps one), row descriptors' record count through readfirstlane: parity, NS A/B
set -o pipefail
OUT=gpurun_out/r06f; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_nosel.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gamma.py tests/test_gpu_parity.py tests/test_big_dag.py tests/test_golden.py > $OUT/pytest_nosel.log 2>&1 || { tail -20 $OUT/pytest_nosel.log; exit 1; }
echo "nosel: $(tail -1 $OUT/pytest_nosel.log)"
bash tools/ab.sh r06f "ns" 2 build/libsk_k17.so build/libsk_nosel.so
