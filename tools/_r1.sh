set -o pipefail
export SK_GIT_HEAD=$1
bash tools/_stamps.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_bpla.py tests/test_bpla_grad.py tests/test_bpla_schedule.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r1_pytest.log 2>&1 || { tail -30 gpurun_out/r1_pytest.log; exit 1; }
tail -1 gpurun_out/r1_pytest.log
bash tools/measure.sh c4 r03n_c4
