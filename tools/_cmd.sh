set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/var_items.log
for cfg in c2 c5; do
for v in base r2; do
  if [ $v = base ]; then L=""; else L=build/libsk_$v.so; fi
  SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "$cfg $v $(tail -1 gpurun_out/vb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_per_launch"])')" >> gpurun_out/var_items.log
done
done
cat gpurun_out/var_items.log
