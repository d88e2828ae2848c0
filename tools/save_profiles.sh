#!/bin/bash
# Copy one tools/measure.sh run (gpurun_out/TAG, merged back from the GPU box)
# into profiles/: the traffic summary the bench reads (profiles/CFG_traffic.json)
# and the round-named evidence (bench line, kernel stats / trace, PMC passes).
# Usage: tools/save_profiles.sh TAG CFG PREFIX   (e.g. r05ns ns r05)
set -e
TAG=$1; CFG=$2; P=$3; OUT=gpurun_out/$TAG
cp $OUT/${CFG}_traffic.json profiles/${CFG}_traffic.json
cp $OUT/${CFG}_traffic.json profiles/${P}_${CFG}_traffic.json
tail -1 $OUT/bench.log > profiles/${P}_${CFG}_bench.json
cp $OUT/prof/run_kernel_stats.csv profiles/${P}_${CFG}_kernel_stats.csv
cp $OUT/prof/run_kernel_trace.csv profiles/${P}_${CFG}_kernel_trace.csv
cp $OUT/FETCH_SIZE/run_counter_collection.csv profiles/${P}_${CFG}_pmc_fetch_size.csv
cp $OUT/WRITE_SIZE/run_counter_collection.csv profiles/${P}_${CFG}_pmc_write_size.csv
cp $OUT/LDS/run_counter_collection.csv profiles/${P}_${CFG}_pmc_lds.csv
ls -la profiles/${P}_${CFG}_*
