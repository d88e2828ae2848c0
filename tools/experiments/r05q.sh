#!/bin/bash
# r05q: stem / string / stem+string cost split at L=200 (N=600: 180k pairs)
set -o pipefail
OUT=gpurun_out/r05q; mkdir -p $OUT; export TMPDIR=/tmp
for k in stem str ss; do
  timeout -k 10 200 python -u tools/probe_perf.py 200 600 $k > $OUT/$k.log 2>&1 || { tail -20 $OUT/$k.log; exit 1; }
  echo "== $k"; grep "pairs/s" $OUT/$k.log | tail -1
done
