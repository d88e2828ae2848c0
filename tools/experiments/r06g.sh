#!/bin/bash
# r06g: select-free IY sweep with the dummy records spread over the free slots (r06f put every
# dummy of a chunk on one slot): parity, NS A/B against the r06e tree, two rounds
set -o pipefail
OUT=gpurun_out/r06g; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libsk_nosel2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_large_configs.py tests/test_gamma.py tests/test_gpu_parity.py tests/test_big_dag.py tests/test_golden.py > $OUT/pytest_nosel2.log 2>&1 || { tail -20 $OUT/pytest_nosel2.log; exit 1; }
echo "nosel2: $(tail -1 $OUT/pytest_nosel2.log)"
bash tools/ab.sh r06g "ns" 2 build/libsk_k17.so build/libsk_nosel2.so
