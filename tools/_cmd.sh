set -o pipefail
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_configs.py tests/test_gamma.py tests/test_gpu_parity.py > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash tools/gpu_quick.sh c2 ns c5 && SK_SERIAL_CLASSES=1 bash tools/gpu_quick.sh c2 ns
