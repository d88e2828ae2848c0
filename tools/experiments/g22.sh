# Whole Grams through sk_gram_sharded on the final tree: C2, C4, C5 (8192 x L300, ~5 min).
set -o pipefail
OUT=gpurun_out/full; mkdir -p $OUT; export TMPDIR=/tmp
for c in c2 c4 c5; do
  timeout -k 10 700 python3 -u bench.py --config $c --full --no-cpu-baseline > $OUT/${c}_full.log 2>&1 || { tail -20 $OUT/${c}_full.log; exit 1; }
  tail -1 $OUT/${c}_full.log | cut -c1-160
done
