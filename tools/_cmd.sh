set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden_ext.py -m gpu > gpurun_out/pytest_gext.log 2>&1 || { tail -30 gpurun_out/pytest_gext.log; exit 1; }
tail -1 gpurun_out/pytest_gext.log
