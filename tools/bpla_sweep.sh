# BPLA kernels: precision probe (general vs fast), parity tests, C4 bench
set -o pipefail
mkdir -p gpurun_out
SK_BPLA_GENERAL=1 timeout -k 5 60 python -u tools/bpla_prec.py 2>&1 | grep -v amdgpu.ids
timeout -k 5 60 python -u tools/bpla_prec.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bpla.py tests/test_large_configs.py -k "bpla or BPLA" -m gpu > gpurun_out/bpla_t.log 2>&1 || { tail -30 gpurun_out/bpla_t.log; exit 1; }
tail -1 gpurun_out/bpla_t.log
for w in ${WAVES:-16}; do
  SK_BPLA_WAVES=$w timeout -k 10 300 python3 -u bench.py --config c4 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_c4_w$w.log 2>&1 || { tail -20 gpurun_out/bench_c4_w$w.log; exit 1; }
  echo -n "waves=$w "; grep '^{' gpurun_out/bench_c4_w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms_per_launch'],3), d['roofline']['launches'])"
done
