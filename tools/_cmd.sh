set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --config c2 > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-100
