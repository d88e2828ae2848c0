set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u tools/probe_perf.py 200 256 stem > gpurun_out/var.log 2>&1 || { tail -20 gpurun_out/var.log; exit 1; }; grep "cycles/row\|pairs/s" gpurun_out/var.log | tail -2; }
for m in 1 14 18 25; do run SK_LIB_PATH=build/libsk_m.so SK_SWEEP_LANES=$m; done
