set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem4d.py tests/test_stem4d_long.py tests/test_large_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for v in 3 4 3 4; do
  export SK4_STREAMS=$v
  timeout -k 10 300 python3 -u bench.py --config c3 --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('c3 streams=$v', round(d['value'],1), d['roofline']['frac'], round(d['ms_per_step'],1))"
done
