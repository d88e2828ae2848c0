set -o pipefail
timeout -k 10 300 python3 -u tools/bpla_dbg.py > gpurun_out/dbg.log 2>&1 || { tail -30 gpurun_out/dbg.log; exit 1; }
tail -6 gpurun_out/dbg.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bpla.py tests/test_golden.py tests/test_bpla_grad.py tests/test_golden_ext.py > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash tools/gpu_quick.sh c4 && SK_BPLA_CHUNK=1 bash tools/gpu_quick.sh c4 && SK_BPLA_CHUNK=8 bash tools/gpu_quick.sh c4
