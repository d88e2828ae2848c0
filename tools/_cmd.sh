set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/probe_perf.py 200 256 stem > gpurun_out/var.log 2>&1 || { tail -20 gpurun_out/var.log; exit 1; }; grep "cycles/row\|pairs/s" gpurun_out/var.log | tail -2; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run SK_LIB_PATH=build/libsk_d0.so
run SK_LIB_PATH=build/libsk_d1.so
run SK_LIB_PATH=build/libsk_d0.so
run SK_LIB_PATH=build/libsk_d1.so
