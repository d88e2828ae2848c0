set -o pipefail
mkdir -p gpurun_out/st
for cfg in "200 512 ss" "300 512 stem"; do
  set -- $cfg
  SK_LIB_PATH=build/libstem_kernel_amd_stamps.so timeout -k 10 200 python -u tools/probe_perf.py $1 $2 $3 > gpurun_out/st/$1_$3.log 2>&1 || { tail -20 gpurun_out/st/$1_$3.log; exit 1; }
  echo "== $cfg"; grep "stamps\|pairs/s" gpurun_out/st/$1_$3.log | tail -7
done
