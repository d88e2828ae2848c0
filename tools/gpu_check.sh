#!/bin/bash
# GPU suite + smoke + one bench line (with CPU baseline and parity) on the
# GPU box.  Usage (through gpurun, repo root): tools/gpu_check.sh TAG [CONFIG]
set -o pipefail
TAG=${1:-chk}; CFG=${2:-ns}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python3 -u bench.py --config $CFG > $OUT/bench_$CFG.log 2>&1 || { tail -20 $OUT/bench_$CFG.log; exit 1; }
tail -1 $OUT/bench_$CFG.log | cut -c1-400
