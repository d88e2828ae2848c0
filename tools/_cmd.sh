set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem4d.py -m gpu > gpurun_out/pytest_s4d.log 2>&1 || { tail -30 gpurun_out/pytest_s4d.log; exit 1; }
tail -1 gpurun_out/pytest_s4d.log
: > gpurun_out/b10.log
for k in stem4d_b10 stem4d_ali stem4d; do
  timeout -k 10 200 python -u tools/probe_perf.py 200 32 $k >> gpurun_out/b10.log 2>&1 || { tail -20 gpurun_out/b10.log; exit 1; }
  echo "== $k" >> gpurun_out/b10.log
done
grep "pairs/s\|==" gpurun_out/b10.log
