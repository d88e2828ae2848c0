set -o pipefail
for v in "" build/libsk_npf20.so "" build/libsk_npf20.so; do
  SK_LIB_PATH=$v timeout -k 10 400 python3 -u bench.py --config ns --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('ns $v', round(d['value']), round(d['roofline']['kernel_ms_per_launch'],1), round(d['ms_per_step'],1))"
done
for v in "" build/libsk_npf12.so "" build/libsk_npf12.so; do
  SK_LIB_PATH=$v timeout -k 10 400 python3 -u bench.py --config c2 --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('c2 $v', round(d['value']), round(d['roofline']['kernel_ms_per_launch'],2), round(d['ms_per_step'],1))"
done
