#!/bin/bash
# r06 final tree: tools/measure.sh for the other SURVEY configs (kernel trace,
# FETCH_SIZE / WRITE_SIZE / LDS passes, bench line) -> profiles/<cfg>_traffic.json
set -o pipefail
for c in c2 c3 c4 c5; do
  bash tools/measure.sh $c r06w_$c || exit 1
  tail -1 gpurun_out/r06w_$c/bench.log | cut -c1-160
done
