#!/bin/bash
# r06 final tree (after the pack / planning / export changes): GPU suite +
# smoke + NS measurement round trip (tools/measure.sh), the default bench command
set -o pipefail
bash tools/measure.sh ns r06t_ns --tests || exit 1
OUT=gpurun_out/r06t_ns; export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-200
