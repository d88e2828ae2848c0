set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gamma.py tests/test_gpu_parity.py tests/test_golden.py tests/test_large_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for cfg in ns c5; do
for v in "" 1 "" 1; do
  if [ -n "$v" ]; then export SK_REF_ORDER=1; else unset SK_REF_ORDER; fi
  SK_PACK_STATS=1 timeout -k 10 400 python3 -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  grep "sk pack" gpurun_out/v.log | tail -1
  python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('$cfg ref_order=$v', round(d['value']), round(d['roofline']['kernel_ms_per_launch'],1), round(d['ms_per_step'],1))"
done
done
