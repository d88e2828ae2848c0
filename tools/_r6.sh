set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_pytest.log 2>&1 || { tail -30 gpurun_out/r6_pytest.log; exit 1; }
tail -1 gpurun_out/r6_pytest.log
bash tools/ab.sh ab6 "c5 ns" 2 - build/libsk_prev.so
