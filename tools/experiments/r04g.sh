#!/bin/bash
# r04g: stall-reason counters of the C3 pre / column kernels, NS DAG and C4 BPLA kernels
set -o pipefail
OUT=gpurun_out/r04g
bash tools/pmc_stall.sh $OUT/c3_pre c3 sk_stem4d_pre && \
bash tools/pmc_stall.sh $OUT/c3_col c3 sk_stem4d_col SK4_COL=1 && \
bash tools/pmc_stall.sh $OUT/ns ns sk_dag_stem_kernel && \
bash tools/pmc_stall.sh $OUT/c4 c4 sk_bpla_fast
