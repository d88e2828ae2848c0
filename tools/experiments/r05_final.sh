#!/bin/bash
# r05 final tree: tools/measure.sh for every config (kernel trace + stats, FETCH / WRITE / LDS passes, bench line)
set -o pipefail
TAG=${1:-r05f}
for c in ${CONFIGS:-ns c3 c2 c4 c5}; do
  tools/measure.sh $c ${TAG}_$c || exit 1
done
