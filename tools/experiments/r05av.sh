#!/bin/bash
# r05av: C3 column kernel on the final r05 tree: stall shares (tools/pmc_stall.sh) and the instruction mix per type
set -o pipefail
OUT=gpurun_out/r05av; mkdir -p $OUT; export TMPDIR=/tmp; ROOT=$(pwd)
tools/pmc_stall.sh $OUT/stall c3 sk_stem4d_col || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVES \
  -d $ROOT/$OUT/mix -o run --output-format csv -- python3 $ROOT/bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/mix.log 2>&1 || { tail -5 $OUT/mix.log; exit 1; }
python3 tools/pmc_sum.py $OUT/mix sk_stem4d_col
