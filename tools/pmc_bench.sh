#!/bin/bash
# HBM traffic of the bench's dominant kernel from rocprofv3 counters, one
# counter per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass), as
# MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes.
# Usage (GPU box): tools/pmc_bench.sh OUTDIR CONFIG [extra bench args]
set -e
OUT=${1:-gpurun_out/pmc_bench}; CFG=${2:-ns}; shift 2 || true
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d $ROOT/$OUT/$c -o run --output-format csv -- \
    python3 $ROOT/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline "$@" \
    > $ROOT/$OUT/$c.log 2>&1
done
echo pmc_done
