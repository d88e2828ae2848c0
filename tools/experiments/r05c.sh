#!/bin/bash
# r05c: stall and instruction counters of the 4-D column kernel (C3 shapes,
# one step of ~514 pairs), one rocprofv3 --pmc pass per counter group
set -o pipefail
TAG=${1:-r05c}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
ARGS="--config c3 --n 256 --slices 64 --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d $ROOT/$OUT/p$i -o run --output-format csv -- python3 $ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  python3 tools/pmc_sum.py $OUT/p$i col_kernel | tee $OUT/p$i.json
done
