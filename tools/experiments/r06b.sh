#!/bin/bash
# r06b: fetch calibration with the Infinity-Cache re-read case; GPU tests of the r06 fixes
# (long x on the 4-D column kernel, per-batch fold tables, column kernel at C3 size)
set -o pipefail
OUT=gpurun_out/r06b; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/calib/run.sh > $OUT/calib.txt 2>&1 || { tail -20 $OUT/calib.txt; exit 1; }
cat $OUT/calib.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_stem4d_long.py tests/test_fold.py tests/test_stem4d.py "tests/test_large_configs.py::test_stem4d_at_config_size" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
