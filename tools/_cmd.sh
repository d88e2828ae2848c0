set -o pipefail
mkdir -p gpurun_out
SK_LIB_PATH=build/libsk_w8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py -m gpu > gpurun_out/pytest_seg.log 2>&1 || { tail -30 gpurun_out/pytest_seg.log; exit 1; }
tail -1 gpurun_out/pytest_seg.log
: > gpurun_out/var_knobs.log
for v in base w8 base w8; do
  if [ $v = base ]; then L=""; else L=build/libsk_$v.so; fi
  SK_LIB_PATH=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/vb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/var_knobs.log
done
cat gpurun_out/var_knobs.log
