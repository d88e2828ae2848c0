#!/bin/bash
# Counter passes for the stem kernel (run on the GPU box).  Usage: tools/pmc_passes.sh OUTDIR L N
set -e
OUT=${1:-gpurun_out/pmc}; L=${2:-200}; N=${3:-128}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d $ROOT/$OUT/p$i -o run --output-format csv -- python3 $ROOT/tools/probe_perf.py $L $N stem > $ROOT/$OUT/p$i.log 2>&1
done
echo passes_done
