set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem4d.py -m gpu -k "long or alignment" > gpurun_out/pytest_s4d.log 2>&1 || { tail -30 gpurun_out/pytest_s4d.log; exit 1; }
tail -4 gpurun_out/pytest_s4d.log
