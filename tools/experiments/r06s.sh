#!/bin/bash
# r06s: GPU suite on the tree with threaded call planning, then the whole NS
# Gram through sk_gram_sharded (bench --full) with SK_HOST_STATS under the
# kernel trace (exposed planning before the first stem launch; r06r: 386 ms plan + 47 ms phi keys)
set -o pipefail
OUT=gpurun_out/r06s; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
SK_HOST_STATS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --full --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
grep "\[host\]\|\[sk upload\]" $OUT/bench.log | tail -5
