set -o pipefail
mkdir -p gpurun_out/r11
SK_HOST_STATS=1 SK_PHI_STATS=1 timeout -k 10 300 python3 -u bench.py --config ns --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r11/ns.log 2>&1 || { tail -20 gpurun_out/r11/ns.log; exit 1; }
grep -E "^\[host\]|^\[phi\]" gpurun_out/r11/ns.log | tail -12
tail -1 gpurun_out/r11/ns.log | cut -c1-400
