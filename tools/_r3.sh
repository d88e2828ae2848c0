set -o pipefail
bash tools/_stamps.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gamma.py tests/test_large_configs.py tests/test_golden.py tests/test_big_dag.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest.log 2>&1 || { tail -30 gpurun_out/r3_pytest.log; exit 1; }
tail -1 gpurun_out/r3_pytest.log
SK_LIB_PATH=$PWD/build/libsk_edg20.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_large_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest20.log 2>&1 || { tail -30 gpurun_out/r3_pytest20.log; exit 1; }
tail -1 gpurun_out/r3_pytest20.log
bash tools/ab.sh ab3 "c5 ns" 2 - build/libsk_edg64.so build/libsk_edg20.so
