#!/bin/bash
# r04i: per-phase cycles of the DAG stem kernel (stamped build) on NS-shaped pairs
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libstem_kernel_amd_stamps.so timeout -k 10 200 python -u tools/probe_perf.py 200 512 stem > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
grep stamps $OUT/stamps.log | tail -12
