#!/bin/bash
# r06h: the MAXK 17 class without its prefetched row (SK_NPF17=0: no spills inside the row loop)
# against one prefetched row (10 spill loads / stores per row), NS A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06h; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab.sh r06h "ns" 2 build/libsk_nosel2.so build/libsk_npf17z.so
