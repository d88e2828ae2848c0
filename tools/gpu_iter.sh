#!/bin/bash
# One development round trip on the GPU box: GPU parity tests, stamped probe,
# plain probe.  Usage: tools/gpu_iter.sh [L] [N]
set -o pipefail
L=${1:-200}; N=${2:-256}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SK_LIB_PATH=build/libstem_kernel_amd_stamps.so timeout -k 10 200 python -u tools/probe_perf.py $L $N stem > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
grep stamps gpurun_out/stamps.log | tail -4
timeout -k 10 200 python -u tools/probe_perf.py $L $N stem > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
tail -2 gpurun_out/probe.log
