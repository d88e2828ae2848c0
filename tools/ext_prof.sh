set -o pipefail
ROOT=$(pwd); OUT=gpurun_out/ext; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/ali -o run --output-format csv -- \
  python3 $ROOT/tools/probe_perf.py 200 32 stem4d_ali > $OUT/ali.log 2>&1 || { tail -20 $OUT/ali.log; exit 1; }
tail -2 $OUT/ali.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/grad -o run --output-format csv -- \
  python3 $ROOT/tools/probe_grad.py 256 > $OUT/grad.log 2>&1 || { tail -20 $OUT/grad.log; exit 1; }
tail -2 $OUT/grad.log
find $OUT -name '*kernel_stats.csv'
