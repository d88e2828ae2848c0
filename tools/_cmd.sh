set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/probe_perf.py 200 256 stem > gpurun_out/var.log 2>&1 || { tail -20 gpurun_out/var.log; exit 1; }; grep "cycles/row\|pairs/s\|class" gpurun_out/var.log | tail -4; }
run SK_LIB_PATH=build/libsk_w12.so
run SK_LIB_PATH=build/libsk_w8n2.so
run SK_LIB_PATH=build/libsk_w8n1.so
