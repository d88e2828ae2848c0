#!/bin/bash
# r06j: the MAXK 16 class without its prefetched row too (SK_NPF16=0) against the r06h winner
# (MAXK 17 without, MAXK 16 with one), NS A/B, two rounds
set -o pipefail
OUT=gpurun_out/r06j; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab.sh r06j "ns" 2 build/libsk_cur.so build/libsk_npf16z.so
