set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bpla or BPLA" > gpurun_out/pytest_bpla.log 2>&1 || { tail -30 gpurun_out/pytest_bpla.log; exit 1; }
tail -1 gpurun_out/pytest_bpla.log
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-200
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_per_launch'])"
