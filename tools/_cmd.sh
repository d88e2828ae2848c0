set -o pipefail
mkdir -p gpurun_out
for cfg in c2 c5 c3; do
  timeout -k 10 400 python3 -u bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || { tail -20 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-120
done
