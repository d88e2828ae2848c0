# A/B of two library builds on C4 (kernel ms per launch, alternating A B A B),
# then the BPLA GPU parity tests on build B (TESTLIB= : the in-tree build).  Usage: bash tools/ab_c4.sh <libB>
set -e
mkdir -p gpurun_out
B=$1
for r in 1 2; do
  for v in A B; do
    lib=""; [ $v = B ] && lib="$PWD/$B"
    SK_LIB_PATH=$lib timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/ab_$v$r.log 2>&1
    echo "$v$r $(tail -1 gpurun_out/ab_$v$r.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["kernel_ms_per_launch"])')" | tee -a gpurun_out/ab_c4.txt
  done
done
SK_LIB_PATH=${TESTLIB-$PWD/$B} timeout -k 10 300 python -u -m pytest tests/test_bpla.py tests/test_large_configs.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
tail -1 gpurun_out/ab_tests.log
