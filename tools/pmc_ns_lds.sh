#!/bin/bash
# LDS / wait counters of the DAG stem kernel on the L=200 probe (512
# examples, SuStem Gram), one rocprofv3 pass per counter group (GPU box).
# Usage: tools/pmc_ns_lds.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc_ns}; mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d $ROOT/$OUT/p$i -o run --output-format csv -- python3 $ROOT/tools/probe_perf.py 200 512 stem > $ROOT/$OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
  python3 tools/pmc_sum.py $OUT/p$i sk_dag_stem_kernel > $OUT/p$i.json || exit 1
  cat $OUT/p$i.json
done
