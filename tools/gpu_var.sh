#!/bin/bash
# Compare library variants on the probe: tools/gpu_var.sh L N lib1.so lib2.so ...
set -o pipefail
L=$1; N=$2; shift 2
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  SK_LIB_PATH=$lib timeout -k 10 200 python -u tools/probe_perf.py $L $N stem > gpurun_out/var.log 2>&1 || { tail -20 gpurun_out/var.log; exit 1; }
  grep "stamps\] classes\|pairs/s" gpurun_out/var.log | tail -2
done
