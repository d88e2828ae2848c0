#!/bin/bash
# r06a: per-phase cycles of the DAG stem kernel (stamped build) on NS-shaped pairs, r06 start
set -o pipefail
OUT=gpurun_out/r06a; mkdir -p $OUT; export TMPDIR=/tmp
SK_LIB_PATH=$PWD/build/libstem_kernel_amd_stamps.so timeout -k 10 200 python -u tools/probe_perf.py 200 512 stem > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
grep stamps $OUT/stamps.log | tail -12
timeout -k 10 200 python -u tools/probe_perf.py 200 512 stem > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 1; }
tail -2 $OUT/plain.log
