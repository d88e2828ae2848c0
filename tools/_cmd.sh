set -o pipefail
timeout -k 10 120 python3 -u tools/str_dbg.py > gpurun_out/sd.log 2>&1 || { tail -5 gpurun_out/sd.log; exit 1; }
tail -2 gpurun_out/sd.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_string_fast.py tests/test_gpu_parity.py tests/test_golden.py tests/test_golden_ext.py > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python3 -u tools/fold_gram_probe.py 2048 200 > gpurun_out/fg.log 2>&1 && tail -3 gpurun_out/fg.log
SK_STR_GENERAL=1 timeout -k 10 300 python3 -u tools/fold_gram_probe.py 2048 200 > gpurun_out/fg2.log 2>&1 && tail -3 gpurun_out/fg2.log
bash tools/gpu_quick.sh ns
