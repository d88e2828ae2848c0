set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c3.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_per_launch'],d['roofline']['launches'],d['ms_per_step'])"
