set -o pipefail
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
SK_HOST_STATS=1 timeout -k 10 300 python3 -u bench.py --config ns --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/hs.log 2>&1; grep -a "\[host\]" gpurun_out/hs.log | tail -2
bash tools/gpu_quick.sh ns
