#!/bin/bash
# C4 instruction counters (one pass, 6 SQ counters) for VALU / SALU / LDS
# instructions per cell; the bench log of the same run gives the cells.
set -e
OUT=${1:-gpurun_out/pmc_c4}
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  -d $ROOT/$OUT/insts -o run --output-format csv -- \
  python3 $ROOT/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $ROOT/$OUT/insts.log 2>&1
echo pmc_done
