#!/bin/bash
# Measurement round trip on the GPU box for one config:
#   GPU parity tests, HBM traffic PMC passes, rocprofv3 kernel stats of the
#   bench, then the plain bench line (with CPU baseline).
# Usage: tools/gpu_bench.sh CONFIG [TAG] [--no-tests]
set -o pipefail
CFG=${1:-ns}; TAG=${2:-$CFG}; NOTESTS=$3
ROOT=$(pwd); OUT=gpurun_out/$TAG
case $CFG in
  ns) KIND=ss; LEN=200; KSUB=sk_dag_stem_kernel;;
  c2) KIND=ss; LEN=150; KSUB=sk_dag_stem_kernel;;
  c5) KIND=stem; LEN=300; KSUB=sk_dag_stem_kernel;;
  c3) KIND=stem4d; LEN=200; KSUB=sk_stem4d_kernel;;
  c4) KIND=bpla; LEN=210; KSUB=sk_bpla;;
esac
mkdir -p $OUT; export TMPDIR=/tmp
if [ "$NOTESTS" != "--no-tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $ROOT/$OUT/$c -o run --output-format csv -- \
    python3 $ROOT/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
done
# traffic per cell -> the box's profiles/ (read by the bench below) and gpurun_out/
python3 tools/pmc_traffic.py $OUT $KSUB $KIND $LEN $OUT/${KIND}_traffic.json > $OUT/traffic.log 2>&1 || { tail -20 $OUT/traffic.log; exit 1; }
cp $OUT/${KIND}_traffic.json profiles/${KIND}_traffic.json
tail -2 $OUT/traffic.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { tail -20 $OUT/bench_prof.log; exit 1; }
timeout -k 10 400 python3 bench.py --config $CFG > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
