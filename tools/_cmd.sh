set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
: > gpurun_out/var_knobs.log
for cfg in ns c5 c2; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/vb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/var_knobs.log
done
cat gpurun_out/var_knobs.log
