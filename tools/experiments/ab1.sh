set -o pipefail
mkdir -p gpurun_out/ab1
SK_PACK_STATS=1 timeout -k 10 300 python3 -u bench.py --config ns --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ab1/pack.log 2>&1 || { tail -20 gpurun_out/ab1/pack.log; exit 1; }
grep "sk pack" gpurun_out/ab1/pack.log
bash tools/ab.sh ab1 "ns c5" 2 - build/libsk_fullstore.so
