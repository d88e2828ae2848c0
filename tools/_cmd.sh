set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/var_items.log
for a in "c5 128" "ns 48" "ns 32"; do
  set -- $a
  timeout -k 10 300 python3 -u bench.py --config $1 --slices $2 --no-cpu-baseline > gpurun_out/vb.log 2>&1 || { tail -20 gpurun_out/vb.log; exit 1; }
  echo "$1 slices=$2 $(tail -1 gpurun_out/vb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" >> gpurun_out/var_items.log
done
cat gpurun_out/var_items.log
