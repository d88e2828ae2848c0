set -o pipefail
mkdir -p gpurun_out/r01_v13
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01_v13/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r01_v13/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r01_v13/pytest_gpu.log
for c in ns c5; do
timeout -k 10 400 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/r01_v13/bench_$c.log 2>&1 || { tail -20 gpurun_out/r01_v13/bench_$c.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r01_v13/bench_$c.log').read().strip().splitlines()[-1]);print('$c',d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_per_launch'])"
done
