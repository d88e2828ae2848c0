set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/var_knobs.log
for v in base npf3 base npf3; do
  if [ $v = base ]; then L=""; else L=build/libsk_$v.so; fi
  SK_LIB_PATH=$L timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/vb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_launch"])')" >> gpurun_out/var_knobs.log
done
cat gpurun_out/var_knobs.log
