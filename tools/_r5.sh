set -o pipefail
bash tools/_stamps.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gamma.py tests/test_large_configs.py tests/test_golden.py tests/test_big_dag.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_pytest.log 2>&1 || { tail -30 gpurun_out/r5_pytest.log; exit 1; }
tail -1 gpurun_out/r5_pytest.log
bash tools/ab.sh ab5 "c5 ns" 2 - build/libsk_pw4.so build/libsk_prev.so
